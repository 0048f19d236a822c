#!/bin/bash
# Ragged default (byte-balanced) + flat IPv4 header kernel: tests, then bench lines 3 and 7.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "ragged or config3 or ipv4 or f3" --timeout 300 --timeout-method thread > gpurun_out/pytest_it3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_it3.log
[ $rc -ne 0 ] && exit $rc
for c in 3 7; do
timeout -k 10 300 python bench.py --config $c --steps 200 --cpu-seconds 0 > gpurun_out/bench_it3_c$c.log 2>&1
rc=$?; echo "bench c$c rc=$rc"; tail -1 gpurun_out/bench_it3_c$c.log | cut -c1-1200
[ $rc -ne 0 ] && exit $rc
done
for k in 0 2; do for b in 2 4 8; do
  timeout -k 10 200 python bench.py --config 7 --steps 100 --cpu-seconds 0 --param kernel=$k --param blocks_per_cu=$b > gpurun_out/c7_k${k}_b$b.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c7_k${k}_b$b.json'));print('kernel=$k bpc=$b', d['kernel_ms_mean'], d['roofline']['frac'])"
done; done
