#!/bin/bash
# Quick GPU check of the current tree: parity tests, smoke, default bench,
# then optional bench configs given as arguments. rc >= 124 ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "gpurun_out/$name.log" | tail -3 | cut -c1-900
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 300 python bench.py
for c in "$@"; do step bench_c$c 300 python bench.py --config $c --steps 100 --cpu-seconds 0; done
