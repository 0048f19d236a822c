#!/bin/bash
# Round 3 (session 2): where the receive pass's prefix form wins — ACK/data mixes (workload
# 17's shape, data_frac varied) and uniform small-to-mid frames (workload 13's shape, hi varied), each form and grid
# in the same process (tools/ab.py).
set -u
out=gpurun_out/${1:-r03q}
mkdir -p "$out"
export TMPDIR=/tmp
V="def:;stream:segs_per_wave=1;lds:segs_per_wave=2;p4:segs_per_wave=3;p3:segs_per_wave=3,blocks_per_cu=3;p2:segs_per_wave=3,blocks_per_cu=2"
for f in ${FRACS:-0.01 0.02 0.1 0.2}; do
  timeout -k 10 200 python tools/ab.py --config 17 --set data_frac=$f --variants "$V" --rounds 5 > "$out/ab_f$f.txt" 2>&1 || exit $?
  grep AB "$out/ab_f$f.txt"
done
for h in ${HIS:-160 250 400 700}; do
  timeout -k 10 200 python tools/ab.py --config 13 --set hi=$h --variants "$V" --rounds 5 > "$out/ab_h$h.txt" 2>&1 || exit $?
  grep AB "$out/ab_h$h.txt"
done
echo done
