#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "tcp_build or f1" --timeout 300 --timeout-method thread > gpurun_out/pytest_it6.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_it6.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/sweep.py --configs 6 --rounds 5 --out gpurun_out/sweep_tcp.json > gpurun_out/sweep_tcp.log 2>&1; echo "sweep6 rc=$?"; grep config6 gpurun_out/sweep_tcp.log | tail -9 | cut -c1-200
