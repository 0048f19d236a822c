#!/bin/bash
# Round 3 pass 12: equal-count wave ranges for batches of small units (mean < 128 B) — receive / ragged parity
# (incl. full-size workloads 13-17 and 15 against the oracle), then alternating library builds against HEAD.
set -u
out=gpurun_out/${1:-r03n}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "small or ragged or rx" > "$out/pytest_focus.log" 2>&1
rc=$?; tail -2 "$out/pytest_focus.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash tools/lib_ab.sh run "13 15 16 17 14 10" 2 > "$out/lib_ab.txt" 2>&1 || exit $?
cat "$out/lib_ab.txt"
echo done
