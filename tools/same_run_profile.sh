#!/bin/bash
# The bench line and its rocprofv3 kernel statistics from ONE command (the measurement contract: the committed
# rocprofv3 --kernel-trace --stats summary is of the same command whose HIP-event kernel time the bench reports).
# usage: tools/same_run_profile.sh <tag> <config...>   → gpurun_out/same_<tag>/c<N>/{bench.json,run_kernel_stats.csv}
set -u
tag=$1; shift
export TMPDIR=/tmp
make -s -j16 -C network-stack_amd || exit 1  # before rocprofv3, never as a child of the profiled process
for c in "$@"; do
  out=gpurun_out/same_${tag}/c$c
  mkdir -p $out
  echo "=== config $c"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run -f csv -- python3 bench.py --config $c --cpu-seconds 0 --no-build > $out/bench.log 2>&1
  rc=$?
  grep '^{' $out/bench.log | tail -1 > $out/bench.json
  find $out -name run_kernel_stats.csv -exec cp {} $out/run_kernel_stats.csv \; 2>/dev/null
  find $out -mindepth 1 -type d -exec rm -rf {} + 2>/dev/null
  echo "=== config $c rc=$rc"; cut -c1-160 $out/bench.json
  if [ $rc -ge 124 ]; then exit $rc; fi
done
