#!/bin/bash
# Build the library from the working tree with extra defines into
# build_var/libbpmx_<name>.so (diagnostic A/B builds; BPMX_LIB selects one).
set -eu
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
d=$root/build_var/src_$name
rm -rf "$d" && mkdir -p "$d/bpm_analysis_amd" "$d/include"
cp -r "$root/bpm_analysis_amd/csrc" "$d/bpm_analysis_amd/"
cp "$root"/include/*.h "$d/include/"
rm -f "$d"/bpm_analysis_amd/csrc/*.o
make -s -j8 -C "$d/bpm_analysis_amd/csrc" OUT="$root/build_var/libbpmx_$name.so" \
  FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function $*"
rm -rf "$d"
echo "built build_var/libbpmx_$name.so"
