#!/bin/bash
# tools/mkv.sh NAME "DEFINES...": build a variant library into ab/NAME (A/B runs);
# MKV_MAKE="VAR=value ..." passes make variables (e.g. SMALL_SCHED=)
set -e
name=$1; shift
d=$PWD/ab/$name
rm -rf "$d"; mkdir -p "$d/lib"
cp -r gr-ldpc_ece535a_amd/ldpc_ece535a "$d/"
rm -rf "$d/ldpc_ece535a/__pycache__"
make -s -C gr-ldpc_ece535a_amd -j8 hip block OUT="$d/lib" $MKV_MAKE \
  HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wall $*" > /dev/null
echo "$name: $*" >> ab/variants.txt
