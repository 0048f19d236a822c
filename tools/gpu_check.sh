#!/bin/bash
# GPU iteration run (one gpurun call): host probe, parity tests, smoke, default
# bench, bench lines for the configs given as arguments, then optional extra
# bench runs.
#   PYTEST_K="ragged"      only the matching -m gpu tests
#   SKIP_TESTS=1 / SKIP_SMOKE=1 / SKIP_BENCH=1
#   TUNE_RUNS="3:rows=16 3:blocks_per_cu=3"   extra bench lines, config:field=v[,field=v]
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
{ nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())";
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-}";
  lscpu | grep -E "Model name|^CPU\(s\)|Thread|Core|Socket"; } > gpurun_out/host.txt 2>&1
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu ${PYTEST_K:+-k "$PYTEST_K"} --timeout 300 --timeout-method thread || exit 1
fi
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
[ "${SKIP_BENCH:-0}" = 1 ] || step bench_c2 300 python bench.py || exit 1
for c in "$@"; do step bench_c$c 300 python bench.py --config $c --steps 100 --cpu-seconds 0 || exit 1; done
i=0
for run in ${TUNE_RUNS:-}; do
  i=$((i+1)); c=${run%%:*}; kv=${run#*:}
  args=(); IFS=',' read -ra parts <<< "$kv"; for p in "${parts[@]}"; do args+=(--tune "$p"); done
  step tune_${i}_c$c 300 python bench.py --config $c --steps 100 --cpu-seconds 0 "${args[@]}" || exit 1
done
