#!/bin/bash
# Round 3 (session 2): the receive pass's kRxBigMean threshold: the default against the
# 15-row prefix form (mode 6) and streamed runs (mode 1) at mean frames of 645-745 B (uniform 40-hi B).
set -u
out=gpurun_out/r03bm
mkdir -p "$out"
export TMPDIR=/tmp
V="def:;p2:segs_per_wave=6;stream:segs_per_wave=1"
for h in 1150 1250 1350 1450; do
  timeout -k 10 200 python tools/ab.py --config 13 --set hi=$h --set n=4194304 --variants "$V" --rounds 5 > "$out/ab_h$h.txt" 2>&1 || exit $?
  grep AB "$out/ab_h$h.txt"
done
echo done
