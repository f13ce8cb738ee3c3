#!/bin/bash
# Same-box A/B of the decode library: builds git revision $1 (A) and the
# working tree (B) into ab/A and ab/B (git-ignored, travels with gpurun),
# then prints the command to run on the box.
#   tools/ab.sh <rev> [bench args]   (here)   ->   bash ab/run.sh   (on the box)
set -e
rev=${1:?rev}; shift
root=$(cd "$(dirname "$0")/.." && pwd)
rm -rf "$root/ab" /tmp/ab_wt && mkdir -p "$root/ab"
git -C "$root" worktree add -f /tmp/ab_wt "$rev" > /dev/null
make -s -j8 -C /tmp/ab_wt/gr-ldpc_ece535a_amd hip
cp -r /tmp/ab_wt/gr-ldpc_ece535a_amd "$root/ab/A"
git -C "$root" worktree remove --force /tmp/ab_wt
make -s -j8 -C "$root/gr-ldpc_ece535a_amd" hip
cp -r "$root/gr-ldpc_ece535a_amd" "$root/ab/B"
args="--no-cpu-baseline --no-variants --no-config4 --no-block --steps 100 --warmup 20 $*"
cat > "$root/ab/run.sh" <<EOS
#!/bin/bash
# alternate A and B three times each; one JSON line per run
for i in 1 2 3; do
  for v in A B; do
    LDPC_PKG_DIR=ab/\$v timeout -k 10 120 python bench.py $args > ab/\$v.\$i.json 2> ab/\$v.\$i.err || exit 1
    python3 -c "import json,sys;d=json.load(open('ab/\$v.\$i.json'));print('\$v', \$i, d['value'], d['timing']['device_span_ms_per_launch'])"
  done
done
EOS
echo "built ab/A ($rev) and ab/B (working tree); run: bash ab/run.sh"
