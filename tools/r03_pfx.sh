#!/bin/bash
# Round 3 (session 2): the receive pass's prefix form. Receive-pass parity (every form,
# the full-size workloads), then same-process A/B of the prefix form's grids against the default forms.
set -u
out=gpurun_out/${1:-r03p}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$out/pytest_rx.log" 2>&1
rc=$?; tail -3 "$out/pytest_rx.log"; [ $rc -eq 0 ] || exit $rc
V="def:;p4:segs_per_wave=3;p3:segs_per_wave=3,blocks_per_cu=3;p2:segs_per_wave=3,blocks_per_cu=2"
for c in ${CFGS:-17 13 16 14 10 11}; do
  timeout -k 10 200 python tools/ab.py --config $c --variants "$V" --rounds 5 > "$out/ab_c$c.txt" 2>&1 || exit $?
  grep AB "$out/ab_c$c.txt"
done
echo done
