#!/bin/bash
# Round-3 GPU pass: the whole -m gpu suite, then bench lines for the headline and the small-frame workloads,
# then a kernel-trace + SQ counter profile of the small-frame receive pass. Every GPU step has its own time
# limit and the steps stop at the first failure.
# usage: tools/r03_gpu_check.sh <tag> [configs...]
set -u
tag=${1:-r03a}; shift || true
cfgs=${*:-"2 13 14 15 16 10"}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1
  rc=$?; tail -3 "$out/pytest_gpu.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
for c in $cfgs; do
  timeout -k 10 240 python -u bench.py --config $c --steps 100 --warmup 10 --cpu-seconds ${CPU_S:-4} \
      > "$out/bench_c$c.json" 2> "$out/bench_c$c.err"
  rc=$?; echo "config $c rc=$rc: $(cut -c1-400 "$out/bench_c$c.json")"; [ $rc -eq 0 ] || exit $rc
done
for c in ${PROF:-}; do
  B="bench.py --config $c --steps 50 --warmup 5 --cpu-seconds 0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_c$c/kt" -o run -f csv -- python3 $B \
      > "$out/prof_c${c}_kt.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d "$out/prof_c$c/sq" -o run -f csv \
      -- python3 $B > "$out/prof_c${c}_sq.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS \
      SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR -d "$out/prof_c$c/sq2" -o run -f csv \
      -- python3 $B > "$out/prof_c${c}_sq2.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$out/prof_c$c/fetch" -o run -f csv \
      -- python3 $B > "$out/prof_c${c}_fetch.log" 2>&1 || exit $?
  echo "profiled config $c"
done
echo done
