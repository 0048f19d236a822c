#!/bin/bash
# Full GPU evidence pass: parity tests, smoke, bench lines for configs 2-5,
# end-to-end host rate, rocprofv3 profiles. Every GPU step has its own limit;
# a timeout/crash (rc >= 124) ends the script.
set -u
tag=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "gpurun_out/$name.log" | tail -3 | cut -c1-600
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
nproc > gpurun_out/host.txt; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Core|Socket" >> gpurun_out/host.txt
step pytest_gpu 900 python -m pytest tests -q -m gpu
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 300 python bench.py
step bench_c3 300 python bench.py --config 3 --cpu-seconds 5
step bench_c4 300 python bench.py --config 4 --steps 50 --cpu-seconds 5
step bench_c5 300 python bench.py --config 5 --steps 20 --cpu-seconds 0
step e2e_host 600 python tools/e2e_host.py
for c in ${PROFILE_CONFIGS:-2 3 4}; do bash tools/profile.sh $c $tag || exit 1; done
