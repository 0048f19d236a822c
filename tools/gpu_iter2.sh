#!/bin/bash
# Ragged balanced-partition iteration: ragged parity tests, then the variant sweep.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "ragged or config3" --timeout 300 --timeout-method thread > gpurun_out/pytest_ragged.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_ragged.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/sweep.py --configs 3 --kind ragged_bal --rounds 5 --out gpurun_out/sweep_ragged_bal.json > gpurun_out/sweep_ragged_bal.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -12 gpurun_out/sweep_ragged_bal.log
