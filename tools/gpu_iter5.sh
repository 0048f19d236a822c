#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "ipv4 or f3" --timeout 300 --timeout-method thread > gpurun_out/pytest_it5.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_it5.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/sweep.py --configs 7 --rounds 7 --out gpurun_out/sweep_ipv4.json > gpurun_out/sweep_ipv4.log 2>&1; echo "sweep7 rc=$?"; grep config7 gpurun_out/sweep_ipv4.log | tail -9 | cut -c1-200
