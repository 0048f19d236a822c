#!/bin/bash
# Bench lines for the f1 / f3 workloads (bench.py --config 6 / 7) + kernel stats.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config 6 --steps 100 --cpu-seconds 5 > gpurun_out/bench_c6.json 2> gpurun_out/bench_c6.err || { tail -20 gpurun_out/bench_c6.err; exit 1; }
cat gpurun_out/bench_c6.json
timeout -k 10 300 python bench.py --config 7 --steps 100 --cpu-seconds 5 > gpurun_out/bench_c7.json 2> gpurun_out/bench_c7.err || { tail -20 gpurun_out/bench_c7.err; exit 1; }
cat gpurun_out/bench_c7.json
