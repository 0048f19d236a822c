#!/bin/bash
# Round 3 pass 14: the receive pass's outer loop loads the next run's offsets one run ahead across switches between
# the streamed and the LDS form: receive parity, then alternating library builds against HEAD.
set -u
out=gpurun_out/${1:-r03p}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > "$out/pytest_rx.log" 2>&1
rc=$?; tail -2 "$out/pytest_rx.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash tools/lib_ab.sh run "17 13 14 10" 3 > "$out/lib_ab.txt" 2>&1 || exit $?
cat "$out/lib_ab.txt"
echo done
