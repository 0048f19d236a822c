#!/bin/bash
# GPU iteration run (one gpurun call): parity tests, smoke, default bench, bench
# lines for the configs given as arguments, then an optional variant sweep.
#   PYTEST_K="ragged"      only the matching -m gpu tests
#   SKIP_TESTS=1 / SKIP_SMOKE=1 / SKIP_BENCH=1
#   SWEEP="--configs 6"    run tools/sweep.py with these arguments at the end
# Every GPU step has its own time limit; a timeout or crash (rc >= 124) ends the
# script, a failing test run ends it too.
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
  return $rc
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu ${PYTEST_K:+-k "$PYTEST_K"} --timeout 300 --timeout-method thread || exit 1
fi
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
[ "${SKIP_BENCH:-0}" = 1 ] || step bench_c2 300 python bench.py || exit 1
for c in "$@"; do step bench_c$c 300 python bench.py --config $c --steps 100 --cpu-seconds 0 || exit 1; done
if [ -n "${SWEEP:-}" ]; then
  step sweep 600 python -u tools/sweep.py $SWEEP --out gpurun_out/sweep.json || exit 1
  grep -E "^config" gpurun_out/sweep.log | grep -v round | cut -c1-220
fi
