#!/bin/bash
# Iteration GPU session: parity tests, then bench + sweep. Each GPU step has
# its own time limit; a crash/timeout ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/log.txt
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/log.txt
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -q -m gpu
step bench 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 2
step sweep 900 python tools/sweep.py --configs ${SWEEP_CONFIGS:-2,3,4} --rounds 3 --iters 10
