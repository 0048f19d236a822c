#!/bin/bash
# Round 3 pass 9: wait counts of the streamed scan loops (nothing in flight at the run loops' entry; 32-bit row
# indices in scan_span; global instead of flat loads in the receive pass's wide-run fallback): receive / ragged
# parity, then alternating library builds against HEAD, then the whole -m gpu suite.
set -u
out=gpurun_out/${1:-r03k}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "small or ragged or rx" > "$out/pytest_focus.log" 2>&1
rc=$?; tail -2 "$out/pytest_focus.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 bash tools/lib_ab.sh run "3 10 11 14 13 15 16" 2 > "$out/lib_ab.txt" 2>&1 || exit $?
cat "$out/lib_ab.txt"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$out/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo done
