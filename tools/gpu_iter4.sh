#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "ipv4 or f3" --timeout 300 --timeout-method thread > gpurun_out/pytest_it4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_it4.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/sweep.py --configs 7 --rounds 5 --out gpurun_out/sweep_ipv4.json > gpurun_out/sweep_ipv4.log 2>&1; echo "sweep7 rc=$?"; grep config7 gpurun_out/sweep_ipv4.log | tail -9 | cut -c1-200
timeout -k 10 300 python -u tools/sweep.py --configs 3 --kind ragged_ab --rounds 15 --out gpurun_out/sweep_ragged_ab.json > gpurun_out/sweep_ragged_ab.log 2>&1; echo "sweep3 rc=$?"; grep config3 gpurun_out/sweep_ragged_ab.log | tail -4 | cut -c1-250
