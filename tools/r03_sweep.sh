#!/bin/bash
# Round 3: blocks per CU against the mean unit size (receive pass and ragged scan), to place the default grid's
# switch between its small- and large-unit block counts.
set -u
out=gpurun_out/${1:-r03f}
mkdir -p "$out"
export TMPDIR=/tmp
ab() {  # ab <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > "$out/ab_$tag.txt" 2>&1
  local rc=$?; echo "== $tag rc=$rc"; grep "^AB" "$out/ab_$tag.txt" | cut -c1-140; [ $rc -eq 0 ] || exit $rc
}
V="b3:blocks_per_cu=3;b4:blocks_per_cu=4;lds4:segs_per_wave=2,blocks_per_cu=4;s1b4:segs_per_wave=1,blocks_per_cu=4"
for hi in 300 400 600 1000; do
  ab rx_hi$hi --config 13 --set hi=$hi --n $((600000000 / (20 + hi / 2))) --variants "$V" --rounds 3
done
R="b2:blocks_per_cu=2;b3:blocks_per_cu=3;b4:blocks_per_cu=4;s4b4:segs_per_wave=4,blocks_per_cu=4"
for hi in 768 1024 1500 3000; do
  ab rg_hi$hi --config 15 --set hi=$hi --n $((900000000 / (32 + hi / 2))) --variants "$R" --rounds 3
done
echo done
