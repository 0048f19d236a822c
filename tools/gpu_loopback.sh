#!/bin/bash
# GPU check of the f2/f4 additions plus config-1 loopback numbers in every mode.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/loopback.jsonl
for m in host batch ring-host ring-gpu; do
  timeout -k 10 120 network-stack_amd/build/nsx_loopback --mode $m --reps 2000 >> gpurun_out/loopback.jsonl 2>&1 || exit 1
done
cat gpurun_out/loopback.jsonl
