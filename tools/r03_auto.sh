#!/bin/bash
# Round 3 (session 2): the receive pass's default grid with in-kernel modes. Receive-pass
# parity, then same-process A/B: the default against each forced mode and the round-3 forms, on the bench workloads
# and on the sweep's mixes.
set -u
out=gpurun_out/${1:-r03a2}
mkdir -p "$out"
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_zz_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "rx" > "$out/pytest_rx.log" 2>&1
rc=$?; tail -3 "$out/pytest_rx.log"; [ $rc -eq 0 ] || exit $rc
fi
V="def:;h4:segs_per_wave=5;p2w:segs_per_wave=6;p2x:segs_per_wave=7;p2:segs_per_wave=3,blocks_per_cu=2;old:blocks_per_cu=4;stream3:segs_per_wave=1"
for c in ${CFGS:-17 13 16 14 10 11}; do
  timeout -k 10 200 python tools/ab.py --config $c --variants "$V" --rounds 5 > "$out/ab_c$c.txt" 2>&1 || exit $?
  grep AB "$out/ab_c$c.txt"
done
for f in ${FRACS:-0.01 0.02 0.1}; do
  timeout -k 10 200 python tools/ab.py --config 17 --set data_frac=$f --variants "$V" --rounds 5 > "$out/ab_f$f.txt" 2>&1 || exit $?
  grep AB "$out/ab_f$f.txt"
done
for h in ${HIS:-160 250 1000 1250}; do
  timeout -k 10 200 python tools/ab.py --config 13 --set hi=$h --variants "$V" --rounds 5 > "$out/ab_h$h.txt" 2>&1 || exit $?
  grep AB "$out/ab_h$h.txt"
done
echo done
