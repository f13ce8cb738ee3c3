#!/bin/bash
# Same-box A/B over build variants x bench arguments.
#   tools/ab_matrix.sh "<common bench args>" "<defines 1>" ... -- "<args A>" "<args B>" ...
# Builds each define set into ab/V<i>/ (as tools/ab_variants.sh) and writes
# ab/runm.sh, which runs every (variant, args) pair twice, interleaved.
set -e
common=$1; shift
defs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do defs+=("$1"); shift; done
shift || true
argsets=("$@")
[ ${#argsets[@]} -eq 0 ] && argsets=("")
root=$(cd "$(dirname "$0")/.." && pwd)
rm -rf "$root/ab" && mkdir -p "$root/ab"
src="$root/gr-ldpc_ece535a_amd"
i=0
for d in "${defs[@]}"; do
  i=$((i + 1))
  mkdir -p "$root/ab/V$i"
  cp -r "$src/ldpc_ece535a" "$root/ab/V$i/"
  make -s -j8 -C "$src" hip OUT="$root/ab/V$i/lib" \
    HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wall $d"
  echo "V$i: $d" >> "$root/ab/variants.txt"
done
{
  echo '#!/bin/bash'
  echo 'cat ab/variants.txt'
  echo 'mkdir -p ab/out'
  echo 'for r in 1 2; do'
  for v in $(seq 1 $i); do
    j=0
    for a in "${argsets[@]}"; do
      j=$((j + 1))
      echo "  LDPC_PKG_DIR=\$PWD/ab/V$v timeout -k 10 200 python bench.py $common $a > ab/out/V$v.A$j.\$r.json 2> gpurun_out/ab_V$v.A$j.\$r.err || { tail -5 gpurun_out/ab_V$v.A$j.\$r.err; exit 1; }"
      echo "  python3 -c \"import json;d=json.load(open('ab/out/V$v.A$j.\$r.json'));print('V$v A$j [$a]', \$r, d['value'], d['timing']['device_span_ms_per_launch'])\""
    done
  done
  echo 'done'
} > "$root/ab/runm.sh"
echo "built $i variants x ${#argsets[@]} arg sets; run: bash ab/runm.sh"
