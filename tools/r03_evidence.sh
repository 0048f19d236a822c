#!/bin/bash
# Round-3 evidence pass on the final tree, in parts that each fit one gpurun call:
#   tools/r03_evidence.sh prof "2 3 10"  — rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes per workload
#                                          (tools/profile.sh, summarised by tools/prof_summary.py into
#                                          gpurun_out/profiles/: r03_config<N>.md, traffic_config<N>.json)
#   tools/r03_evidence.sh bench          — -m gpu suite, smoke, every bench line with its CPU legs, host end to end,
#                                          config-1 loopback (tools/gpu_round.sh's steps)
#   tools/r03_evidence.sh same "2 3"     — each bench line under rocprofv3 --kernel-trace --stats (one command)
# Every GPU step has its own limit; a timeout or crash (rc >= 124) ends the script.
set -u
mode=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/r03ev
step() {  # step <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r03ev/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "gpurun_out/r03ev/$name.log" | tail -2 | cut -c1-400
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
case $mode in
  prof)
    mkdir -p gpurun_out/profiles
    for c in ${1:-2 3 10 11 13 14 15 16 17 18}; do
      GROUPS_ONLY="kt fetch write" bash tools/profile.sh $c r03 || exit 1
      python3 tools/prof_summary.py r03 $c > /dev/null || exit 1
      cp profiles/r03_config${c}.md profiles/r03_config${c}_kernel_stats.csv profiles/traffic_config${c}.json \
        gpurun_out/profiles/ || exit 1
      rm -rf gpurun_out/prof_r03_c${c}
      echo "profiled config $c"
    done
    ;;
  bench)  # tools/r03_evidence.sh bench "tests 2 3 ..." — "tests" runs the -m gpu suite and smoke first
    { nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())";
      cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-}";
      lscpu | grep -E "Model name|^CPU\(s\)|Thread|Core|Socket"; } > gpurun_out/r03ev/host.txt 2>&1
    for c in ${1:-tests 2 3 4 5 6 7 8 9 10 11 12 13 14 15 16 17 18}; do
      case $c in
        tests) step pytest_gpu 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider
               step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        2) step bench_c2 300 python bench.py ;;
        3) step bench_c3 300 python bench.py --config 3 --cpu-seconds 5 ;;
        4|12) step bench_c$c 300 python bench.py --config $c --steps 50 --cpu-seconds 5 ;;
        5) step bench_c5 300 python bench.py --config 5 --steps 20 --cpu-seconds 0 ;;
        *) step bench_c$c 300 python bench.py --config $c --steps 100 --cpu-seconds 5 ;;
      esac
    done
    ;;
  host)
    step e2e_host 600 python tools/e2e_host.py
    rm -f gpurun_out/r03ev/loopback.jsonl
    for m in host batch ring-host ring-gpu; do
      step loopback_$m 120 network-stack_amd/build/nsx_loopback --mode $m --reps 2000
      cat gpurun_out/r03ev/loopback_$m.log >> gpurun_out/r03ev/loopback.jsonl
    done
    ;;
  same)
    bash tools/same_run_profile.sh r03 ${1:-2 3 4 5 6 7 8 9 10 11 12 13 14 15 16 17 18} || exit $?
    ;;
esac
echo done
