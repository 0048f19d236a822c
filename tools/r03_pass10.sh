#!/bin/bash
# Round 3 pass 10: lds_range_sum with 4-chunk follow-up blocks (was 8): small-frame / ragged parity, then
# alternating library builds against HEAD on the LDS-form workloads.
set -u
out=gpurun_out/${1:-r03l}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "small or ragged or rx" > "$out/pytest_focus.log" 2>&1
rc=$?; tail -2 "$out/pytest_focus.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/lib_ab.sh run "15 13 16 14" 3 > "$out/lib_ab.txt" 2>&1 || exit $?
cat "$out/lib_ab.txt"
echo done
