#!/bin/bash
# Build libbpmx.so from a git revision (default HEAD) into build_var/libbpmx_<name>.so,
# for A/B runs against the working tree (tools/ab_quick.sh; BPMX_LIB selects a build).
set -eu
rev=${1:-HEAD}; name=${2:-head}
root=$(cd "$(dirname "$0")/.." && pwd)
d=$(mktemp -d /tmp/bpmx_ref.XXXXXX)
git -C "$root" archive "$rev" bpm_analysis_amd/csrc include | tar -x -C "$d"
rm -f "$d"/bpm_analysis_amd/csrc/*.o
mkdir -p "$root/build_var"
make -s -j8 -C "$d/bpm_analysis_amd/csrc" OUT="$root/build_var/libbpmx_$name.so"
rm -rf "$d"
echo "built build_var/libbpmx_$name.so from $rev"
