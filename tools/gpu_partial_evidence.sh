#!/bin/bash
# Evidence for a subset of workloads after a kernel change: GPU suite, PMC traffic + rocprofv3 summaries,
# bench lines with CPU baselines, and the same-command bench + rocprofv3 statistics.
#   bash tools/gpu_partial_evidence.sh <tag> "<configs>"
set -u
tag=$1; configs=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
PROFILE_CONFIGS="$configs" bash tools/gpu_profiles.sh $tag || exit 1
for c in $configs; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --cpu-seconds 5 > gpurun_out/bench_c$c.log 2>&1 || exit 1
  echo "bench $c: $(tail -1 gpurun_out/bench_c$c.log | cut -c1-120)"
done
bash tools/same_run_profile.sh $tag $configs
