#!/bin/bash
# Instruction counts of one workload's kernel under two or more library builds (SQ_INSTS_VALU
# before/after): each build is swapped into network-stack_amd/lib/ in turn (restored on exit) and profiled by
# tools/profile.sh's kt, sq and sq2 passes; tools/valu_ab.py tabulates the per-launch counters.
#   bash tools/valu_ab.sh 13 "r04 new"     # new = the working tree's build; x = network-stack_amd/lib_x/libnsx_csum.so
set -u
cd "$(dirname "$0")/.."
cfg=${1:-13}; libs=${2:-r04 new}
make -s -j16 -C network-stack_amd || exit 1
lib=network-stack_amd/lib/libnsx_csum.so
cp "$lib" /tmp/valu_ab_new.so
trap 'cp /tmp/valu_ab_new.so "$lib"' EXIT
for k in $libs; do
  if [ "$k" = new ]; then cp /tmp/valu_ab_new.so "$lib"; else cp "network-stack_amd/lib_$k/libnsx_csum.so" "$lib"; fi
  NO_MAKE=1 GROUPS_ONLY="kt sq sq2" bash tools/profile.sh "$cfg" "valu_$k" || exit $?
done
