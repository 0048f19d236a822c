#!/bin/bash
# GPU evidence pass, part 1: parity tests, smoke, bench lines for configs 2-9,
# end-to-end host rate, config-1 loopback. Part 2 (profiles) is
# tools/gpu_profiles.sh. Every GPU step has its own limit; a timeout/crash
# (rc >= 124) ends the script.
set -u
tag=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
SKIP_TESTS=${SKIP_TESTS:-0}
step() {  # step <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "gpurun_out/$name.log" | tail -3 | cut -c1-600
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
{ nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())";
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-}";
  lscpu | grep -E "Model name|^CPU\(s\)|Thread|Core|Socket"; } > gpurun_out/host.txt 2>&1
[ "$SKIP_TESTS" = 1 ] || step pytest_gpu 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 300 python bench.py
step bench_c3 300 python bench.py --config 3 --cpu-seconds 5
step bench_c4 300 python bench.py --config 4 --steps 50 --cpu-seconds 5
step bench_c5 300 python bench.py --config 5 --steps 20 --cpu-seconds 0
step bench_c6 300 python bench.py --config 6 --steps 100 --cpu-seconds 5
step bench_c7 300 python bench.py --config 7 --steps 100 --cpu-seconds 5
step bench_c8 300 python bench.py --config 8 --steps 100 --cpu-seconds 5
step bench_c9 300 python bench.py --config 9 --steps 100 --cpu-seconds 5
step bench_c10 300 python bench.py --config 10 --steps 100 --cpu-seconds 5
step bench_c11 300 python bench.py --config 11 --steps 100 --cpu-seconds 5
step bench_c12 300 python bench.py --config 12 --steps 50 --cpu-seconds 5
step e2e_host 600 python tools/e2e_host.py
rm -f gpurun_out/loopback.jsonl
for m in host batch ring-host ring-gpu; do
  step loopback_$m 120 network-stack_amd/build/nsx_loopback --mode $m --reps 2000
  cat gpurun_out/loopback_$m.log >> gpurun_out/loopback.jsonl
done
