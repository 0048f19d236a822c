#!/bin/bash
# Round 3: the receive pass's LDS form — parity first (receive-pass tests + the rx fuzz), then same-process
# A/B of the forms on the small-frame workloads and on mixes around the crossover.
set -u
out=gpurun_out/${1:-r03b}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_zz_fuzz.py tests/test_gpu_parity.py \
    tests/test_gpu_00_baseline.py -k "rx or ragged or config3" -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/pytest_rx.log" 2>&1
rc=$?; tail -3 "$out/pytest_rx.log"; [ $rc -eq 0 ] || exit $rc
ab() {  # ab <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > "$out/ab_$tag.txt" 2>&1
  local rc=$?; echo "== $tag rc=$rc"; tail -6 "$out/ab_$tag.txt"; [ $rc -eq 0 ] || exit $rc
}
V="auto:;lds:segs_per_wave=2;s4:segs_per_wave=4;s1:segs_per_wave=1"
ab c13 --config 13 --variants "$V" --rounds 5
ab c16 --config 16 --variants "$V" --rounds 5
for hi in 160 220 300 500; do
  ab c13_hi$hi --config 13 --set hi=$hi --n $((560000000 / (20 + hi))) --variants "$V" --rounds 5
done
ab c10 --config 10 --variants "$V" --rounds 5
ab c15 --config 15 --variants "$V" --rounds 5
ab c3 --config 3 --variants "$V" --rounds 5
ab c14 --config 14 --variants "$V" --rounds 5
echo done
