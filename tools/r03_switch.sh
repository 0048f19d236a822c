#!/bin/bash
# Round 3 (session 2): the default grid's small-frame mode as the LDS loop that hands over to the hybrid loop at the
# first run needing it: receive-pass parity, then same-process A/B against the hybrid loop
# throughout (mode 7) on ACK-only batches and ACK mixes with a few full frames.
set -u
out=gpurun_out/${1:-r03sw}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_zz_fuzz.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "rx" > "$out/pytest.log" 2>&1
rc=$?; tail -3 "$out/pytest.log"; [ $rc -eq 0 ] || exit $rc
V="def:;hyb:segs_per_wave=7;old:blocks_per_cu=4"
for c in 13 16; do
  timeout -k 10 200 python tools/ab.py --config $c --variants "$V" --rounds 7 > "$out/ab_c$c.txt" 2>&1 || exit $?
  grep AB "$out/ab_c$c.txt"
done
for f in 0.002 0.01 0.02; do
  timeout -k 10 200 python tools/ab.py --config 17 --set data_frac=$f --variants "$V" --rounds 5 > "$out/ab_f$f.txt" 2>&1 || exit $?
  grep AB "$out/ab_f$f.txt"
done
timeout -k 10 200 python tools/ab.py --config 13 --set hi=160 --variants "$V" --rounds 5 > "$out/ab_h160.txt" 2>&1 || exit $?
grep AB "$out/ab_h160.txt"
echo done
