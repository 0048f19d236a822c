#!/bin/bash
# First GPU session: parity tests, smoke, bench, sweep. Each GPU step has its
# own time limit; a crash/timeout (exit >= 124 or signal) ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/log.txt
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/log.txt
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -ge 128 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
rocminfo | grep -m2 -E "gfx950|Marketing" > gpurun_out/rocminfo.txt 2>&1 || true
nproc > gpurun_out/host.txt; lscpu | grep -E "Model name|^CPU\(s\)" >> gpurun_out/host.txt
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -q -m gpu
step bench 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 5
step sweep 600 python tools/sweep.py --configs 2,3,4 --rounds 3 --iters 10
