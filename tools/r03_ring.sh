#!/bin/bash
# Round 3: the receive pass's header windows from an LDS ring — parity, then new vs base
# library in alternating processes, FETCH_SIZE of workload 10, then the blocks-per-CU sweep.
set -u
out=gpurun_out/${1:-r03g}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_zz_fuzz.py -k "rx" -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/pytest_rx.log" 2>&1
rc=$?; tail -2 "$out/pytest_rx.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/lib_ab.sh run "10 11 14" 3 > "$out/lib_ab.txt" 2>&1; rc=$?; cat "$out/lib_ab.txt" | cut -c1-120
[ $rc -eq 0 ] || exit $rc
B="bench.py --config 10 --steps 50 --warmup 5 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$out/fetch10" -o run -f csv -- python3 $B \
    > "$out/fetch10.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/kt10" -o run -f csv -- python3 $B > "$out/kt10.log" 2>&1 || exit $?
bash tools/r03_sweep.sh ${1:-r03g}
