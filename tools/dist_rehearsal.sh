#!/bin/bash
# Multi-rank rehearsal of bench.py on a 1-GPU box: torchrun with N ranks over gloo, all ranks on cuda:0
# (NSX_BENCH_BACKEND=gloo). Exercises the contract's N>1 path end to end: rendezvous at 127.0.0.1, per-rank
# seeds, barrier-bracketed timing, max over ranks, whole-job value. Usage: tools/dist_rehearsal.sh [N]
set -u
n=${1:-2}
mkdir -p gpurun_out
# no make here: the ranks torchrun starts bring the library up to date themselves, the first under bench.py's file
# lock and the rest finding nothing to do; touching a source first makes the first rank really build
[ -n "${TOUCH_SRC:-}" ] && touch network-stack_amd/csrc/host_csum.cpp
stamp() { echo "$1: $(stat -c '%y' network-stack_amd/lib/libnsx_csum.so)"; }
stamp "library before" > gpurun_out/dist_rehearsal_n$n.stamps
NSX_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus "$n" --steps 50 --warmup 5 \
  > gpurun_out/dist_rehearsal_n$n.log 2>&1
rc=$?
stamp "library after" >> gpurun_out/dist_rehearsal_n$n.stamps
cat gpurun_out/dist_rehearsal_n$n.stamps
grep -v amdgpu.ids gpurun_out/dist_rehearsal_n$n.log | tail -3 | cut -c1-700
exit $rc
