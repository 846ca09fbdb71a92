#!/bin/bash
# Build the library from a git revision (default HEAD) into
# build_var/libbpmx_<name>.so, for A/B runs against the working tree.
set -eu
rev=${1:-HEAD}; name=${2:-head}
root=$(cd "$(dirname "$0")/.." && pwd)
d=$root/build_var/src_$name
rm -rf "$d" && mkdir -p "$d"
git -C "$root" archive "$rev" bpm_analysis_amd/csrc include | tar -x -C "$d"
make -s -j8 -C "$d/bpm_analysis_amd/csrc" OUT="$root/build_var/libbpmx_$name.so"
rm -rf "$d"
echo "built build_var/libbpmx_$name.so from $rev"
