#!/bin/bash
# Round 3 pass 4: parity, then the LDS forms with unclamped chunk reads and the 4-blocks/CU receive kernel
# (register-capped at 128 VGPRs), and the LDS-staging probe on config 2.
set -u
out=gpurun_out/${1:-r03d}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_zz_fuzz.py tests/test_gpu_parity.py \
    -k "rx or ragged" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/pytest_rx.log" 2>&1
rc=$?; tail -2 "$out/pytest_rx.log"; [ $rc -eq 0 ] || exit $rc
ab() {  # ab <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > "$out/ab_$tag.txt" 2>&1
  local rc=$?; echo "== $tag rc=$rc"; grep "^AB" "$out/ab_$tag.txt" | cut -c1-140; [ $rc -eq 0 ] || exit $rc
}
V="auto:;b4:blocks_per_cu=4;lds4:segs_per_wave=2,blocks_per_cu=4;s1b4:segs_per_wave=1,blocks_per_cu=4;s4:segs_per_wave=4"
ab c13 --config 13 --variants "$V" --rounds 5
ab c16 --config 16 --variants "$V" --rounds 5
ab c10 --config 10 --variants "$V" --rounds 5
ab c11 --config 11 --variants "$V" --rounds 5
ab c14 --config 14 --variants "$V" --rounds 5
ab c13_hi220 --config 13 --set hi=220 --n 2333333 --variants "$V" --rounds 5
R="auto:;b3:blocks_per_cu=3;b4:blocks_per_cu=4;s4:segs_per_wave=4;s4b4:segs_per_wave=4,blocks_per_cu=4"
ab c15 --config 15 --variants "$R" --rounds 5
ab c15_hi256 --config 15 --set hi=256 --n 4375000 --variants "$R" --rounds 5
ab c3 --config 3 --variants "$R" --rounds 5
timeout -k 10 120 tools/probes/lds_stage > "$out/lds_stage.txt" 2>&1; rc=$?; cat "$out/lds_stage.txt"; [ $rc -eq 0 ] || exit $rc
echo done
