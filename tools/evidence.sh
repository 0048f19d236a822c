#!/bin/bash
# The evidence runs of a round, one parametrised script (round 4 folded round 3's ~35 one-off tools/r03_*.sh
# into these modes). Each mode fits one gpurun call; every GPU step has its own time limit, and a timeout or
# crash (rc >= 124) ends the script with nothing else started on the GPU.
#
#   TAG=r04 tools/evidence.sh host                   — host record: CPUs, cgroup quota, OMP, `go version`, rocm-smi
#   TAG=r04 tools/evidence.sh tests                  — the -m gpu suite, then smoke()
#   TAG=r04 tools/evidence.sh bench "2 2n 3 ..."     — bench lines (2n = config 2 with --no-pseudo)
#   TAG=r04 tools/evidence.sh prof "2 2n 15"         — rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes per
#                                                      workload (tools/profile.sh → tools/prof_summary.py)
#   TAG=r04 tools/evidence.sh sq "15 13"             — SQ instruction-mix / wait counters (profile.sh groups sq, sq2)
#   TAG=r04 tools/evidence.sh ab <config> "<variants>" [ab.py args...]
#                                                    — same-process A/B of nsx_tune launch shapes (tools/ab.py)
#   TAG=r04 tools/evidence.sh sweep <config> "<variants>" "<k=v1 v2 ...>" [ab.py args...]
#                                                    — the same A/B at every value of one workload field
#                                                      (e.g. "hi=1150 1250 1350")
#   TAG=r04 tools/evidence.sh libab "15 3" [pairs]   — the working tree's library against lib_base (tools/lib_ab.sh)
#   TAG=r04 tools/evidence.sh same "2 3"             — each bench line under rocprofv3 --kernel-trace --stats
#   TAG=r04 tools/evidence.sh e2e                    — host memory end to end + the config-1 loopback modes
set -u
mode=$1; shift
tag=${TAG:-r04}
out=gpurun_out/$tag
export TMPDIR=/tmp
mkdir -p "$out"
step() {  # step <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "$out/$name.log" | tail -2 | cut -c1-600
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
  return $rc
}
bench_args() {  # bench_args <workload> → bench.py arguments (Nn = workload N with --no-pseudo)
  local c=${1%n} extra=""
  [ "$c" != "$1" ] && extra="--no-pseudo"
  case $c in
    2) echo "--config 2 $extra" ;;
    3) echo "--config 3 --cpu-seconds 5 $extra" ;;
    4|12) echo "--config $c --steps 50 --cpu-seconds 5 $extra" ;;
    5) echo "--config 5 --steps 20 --cpu-seconds 0 $extra" ;;
    *) echo "--config $c --steps 100 --cpu-seconds 5 $extra" ;;
  esac
}
case $mode in
  host)
    { echo "# $(date -u +%FT%TZ) $(hostname)"; nproc
      python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"
      echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-}"
      lscpu | grep -E "Model name|^CPU\(s\)|Thread|Core|Socket"
      echo "--- go toolchain (SURVEY.md §8d: time a committed Go restatement if one exists)"
      echo "which go: $(which go 2>&1 || echo 'not found')"; echo "go version: $(go version 2>&1)"
      echo "which gccgo: $(which gccgo 2>&1 || echo 'not found')"; ls -d /usr/local/go /usr/lib/go* 2>&1
      echo "--- gpu"; rocm-smi --showproductname --showbus 2>&1 | grep -v "^$" | head -20
      echo "--- make -q (is the pushed library up to date with its sources here?)"
      make -q -C network-stack_amd lib/libnsx_csum.so && echo "up to date" || echo "would rebuild"
    } > "$out/host.txt" 2>&1
    cat "$out/host.txt"
    ;;
  tests)
    step pytest_gpu 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
    ;;
  bench)
    for c in ${1:-2 2n 3 4 5 6 7 8 9 10 11 12 13 14 15 16 17 18}; do
      step bench_c$c 300 python bench.py $(bench_args $c) || exit $?
      grep '^{' "$out/bench_c$c.log" > "$out/bench_c$c.json"
    done
    ;;
  prof)
    mkdir -p gpurun_out/profiles
    for c in ${1:-2 3 15}; do
      n=${c%n}; x=""; [ "$n" != "$c" ] && x="--no-pseudo"
      BENCH_EXTRA="$x" GROUPS_ONLY="kt fetch write" bash tools/profile.sh $n $tag $c || exit 1
      python3 tools/prof_summary.py $tag $c > /dev/null || exit 1
      cp profiles/${tag}_config${c}.md profiles/${tag}_config${c}_kernel_stats.csv profiles/traffic_config${c}.json \
        gpurun_out/profiles/ || exit 1
      rm -rf gpurun_out/prof_${tag}_c${c}
      echo "profiled config $c"
    done
    ;;
  sq)
    for c in ${1:-15 13}; do
      GROUPS_ONLY="sq sq2" bash tools/profile.sh $c ${tag}sq || exit 1
    done
    ;;
  ab)
    c=$1; v=$2; shift 2
    step ab_c$c 600 python tools/ab.py --config $c --variants "$v" "$@" || exit $?
    grep AB "$out/ab_c$c.log"
    ;;
  sweep)
    c=$1; v=$2; kv=$3; shift 3
    k=${kv%%=*}
    for x in ${kv#*=}; do
      step ab_c${c}_$k$x 300 python tools/ab.py --config $c --set $k=$x --variants "$v" "$@" || exit $?
      grep AB "$out/ab_c${c}_$k$x.log" | sed "s/^/$k=$x /"
    done
    ;;
  libab)
    step libab 1200 bash tools/lib_ab.sh run "${1:-2}" "${2:-2}" || exit $?
    cat "$out/libab.log"
    ;;
  same)
    bash tools/same_run_profile.sh $tag ${1:-2 3 15} || exit $?
    ;;
  e2e)
    step e2e_host 600 python tools/e2e_host.py || exit $?
    rm -f "$out/loopback.jsonl"
    for m in host batch ring-host ring-gpu; do
      step loopback_$m 120 network-stack_amd/build/nsx_loopback --mode $m --reps 2000 || exit $?
      cat "$out/loopback_$m.log" >> "$out/loopback.jsonl"
    done
    ;;
  *)
    sed -n '2,25p' "$0"; exit 2 ;;
esac
echo done
