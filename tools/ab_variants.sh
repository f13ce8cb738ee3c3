#!/bin/bash
# Builds the working tree's decode library once per variant (extra hipcc
# defines) into ab/V<i>/ and writes ab/runv.sh, which benches each variant in
# turn (twice) on the GPU box.
#   tools/ab_variants.sh "<bench args>" "<defines 1>" "<defines 2>" ...
# A variant "@<git rev>" builds that revision instead (e.g. "@HEAD").
set -e
args=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
rm -rf "$root/ab" && mkdir -p "$root/ab"
i=0
for defs in "$@"; do
  i=$((i + 1))
  mkdir -p "$root/ab/V$i"
  src="$root/gr-ldpc_ece535a_amd"
  if [[ "$defs" == @* ]]; then  # "@<git rev>": that revision's library, default flags
    rm -rf /tmp/ab_wt && git -C "$root" worktree add -f /tmp/ab_wt "${defs#@}" > /dev/null
    src=/tmp/ab_wt/gr-ldpc_ece535a_amd
    cp -r "$src/ldpc_ece535a" "$root/ab/V$i/"
    make -s -j8 -C "$src" hip OUT="$root/ab/V$i/lib"
    git -C "$root" worktree remove --force /tmp/ab_wt
  else
    # "<defines>|<make variables>", e.g. "-DLDPC_TP_MINB=3" or "|SMALL_SCHED="
    mvars=""
    if [[ "$defs" == *"|"* ]]; then mvars=${defs#*|}; fi
    cp -r "$src/ldpc_ece535a" "$root/ab/V$i/"
    make -s -j8 -C "$src" hip OUT="$root/ab/V$i/lib" $mvars \
      HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wall ${defs%%|*}"
  fi
  echo "V$i: $defs" >> "$root/ab/variants.txt"
done
cat > "$root/ab/runv.sh" <<EOS
#!/bin/bash
cat ab/variants.txt
mkdir -p ab/out
for r in 1 2; do
  for d in ab/V[0-9]*/; do
    d=\${d%/}
    v=\$(basename \$d)
    LDPC_PKG_DIR=\$PWD/\$d timeout -k 10 200 python bench.py $args > ab/out/\$v.\$r.json 2> gpurun_out/ab_\$v.\$r.err || { tail -5 gpurun_out/ab_\$v.\$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('ab/out/\$v.\$r.json'));print('\$v', \$r, d['value'], d['timing']['device_span_ms_per_launch'])"
  done
done
EOS
echo "built $i variants; run: bash ab/runv.sh"
