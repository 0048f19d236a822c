#!/bin/bash
# Round 3 pass 5: parity, then the default grids that pick their active blocks by the batch's mean unit
# (4 blocks/CU for small frames/segments, 3 / 2 for large) against fixed grids.
set -u
out=gpurun_out/${1:-r03e}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_zz_fuzz.py tests/test_gpu_parity.py \
    tests/test_gpu_00_baseline.py -k "rx or ragged or config3" -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$out/pytest_rx.log" 2>&1
rc=$?; tail -2 "$out/pytest_rx.log"; [ $rc -eq 0 ] || exit $rc
ab() {  # ab <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > "$out/ab_$tag.txt" 2>&1
  local rc=$?; echo "== $tag rc=$rc"; grep "^AB" "$out/ab_$tag.txt" | cut -c1-140; [ $rc -eq 0 ] || exit $rc
}
V="auto:;b3:blocks_per_cu=3;b4:blocks_per_cu=4"
for c in 10 11 14 13 16; do ab c$c --config $c --variants "$V" --rounds 5; done
ab c13_hi220 --config 13 --set hi=220 --n 2333333 --variants "$V;lds4:segs_per_wave=2,blocks_per_cu=4" --rounds 5
R="auto:;b2:blocks_per_cu=2;b3:blocks_per_cu=3;b4:blocks_per_cu=4"
ab c3 --config 3 --variants "$R" --rounds 5
ab c15 --config 15 --variants "$R" --rounds 5
ab c15_hi256 --config 15 --set hi=256 --n 4375000 --variants "$R;s4b4:segs_per_wave=4,blocks_per_cu=4" --rounds 5
ab c15_hi512 --config 15 --set hi=512 --n 2430555 --variants "$R;s4b4:segs_per_wave=4,blocks_per_cu=4" --rounds 5
echo done
