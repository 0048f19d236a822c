#!/bin/bash
# Round 3 (session 2): parity of the generic prefix loop (receive pass and ragged checksum), A/B of the receive
# pass's small-frame workloads against the round-3 LDS form, and the ragged checksum's forms over segment sizes.
set -u
out=gpurun_out/${1:-r03a3}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_parity.py tests/test_gpu_zz_fuzz.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider -k "rx or ragged or prefix" > "$out/pytest.log" 2>&1
rc=$?; tail -3 "$out/pytest.log"; [ $rc -eq 0 ] || exit $rc
V="def:;old:blocks_per_cu=4"
for c in 13 16 17; do
  timeout -k 10 200 python tools/ab.py --config $c --variants "$V" --rounds 7 > "$out/ab_c$c.txt" 2>&1 || exit $?
  grep AB "$out/ab_c$c.txt"
done
V="def:;h5:segs_per_wave=5;w6:segs_per_wave=6;p4:segs_per_wave=3;p3:segs_per_wave=3,blocks_per_cu=3;four:segs_per_wave=4"
for h in 128 250 500 1000 2000; do
  timeout -k 10 200 python tools/ab.py --config 15 --set hi=$h --variants "$V" --rounds 5 > "$out/ab_r$h.txt" 2>&1 || exit $?
  grep AB "$out/ab_r$h.txt"
done
timeout -k 10 200 python tools/ab.py --config 3 --variants "$V" --rounds 5 > "$out/ab_c3.txt" 2>&1 || exit $?
grep AB "$out/ab_c3.txt"
echo done
