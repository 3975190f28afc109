#!/bin/bash
# Build the library of a git revision as vproxy_amd/libvpcsum_ab.so (the "old" side of
# tools/ab_libs.sh / ab_libs_cold.sh / ab_nat.sh), on the CPU.  usage: tools/build_ab.sh <rev>
set -euo pipefail
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
T=$(mktemp -d)
git archive "$REV" vproxy_amd include | tar -x -C "$T"
python "$T/vproxy_amd/build.py" --force > /dev/null 2>&1
cp "$T/vproxy_amd/libvpcsum.so" vproxy_amd/libvpcsum_ab.so
rm -rf "$T"
echo "vproxy_amd/libvpcsum_ab.so <- $(git rev-parse --short "$REV")"
