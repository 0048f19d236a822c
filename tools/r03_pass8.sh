#!/bin/bash
# Round 3 pass 8: the LDS loops entered with nothing in flight (no per-run vmcnt(0) on result stores):
# small-frame and ragged parity, then alternating library builds against the same tree without the entry wait,
# then SQ counters of workload 13 (instructions and waits per 64-frame run).
set -u
out=gpurun_out/${1:-r03j}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "small or ragged or rx" > "$out/pytest_focus.log" 2>&1
rc=$?; tail -2 "$out/pytest_focus.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash tools/lib_ab.sh run "13 15 16 14 10 11 3" 2 > "$out/lib_ab.txt" 2>&1 || exit $?
cat "$out/lib_ab.txt"
B="bench.py --config 13 --steps 50 --warmup 5 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT -d "$out/pmc13" -o run -f csv \
    -- python3 $B > "$out/pmc13.log" 2>&1 || exit $?
echo done
