#!/bin/bash
# Config 5's span effect: address-translation and L2 counters for one 25 GB launch
# against the default back-to-back ~1.6 GB windows. One --pmc pass per counter group.
set -u
export TMPDIR=/tmp
out=gpurun_out/c5_span; mkdir -p $out
make -s -j16 -C network-stack_amd || exit 1  # before rocprofv3; bench.py then loads it as it is
for v in windows one; do
  T=""; [ $v = one ] && T="--tune window_bytes=-1"
  B="bench.py --config 5 --steps 6 --warmup 2 --settle-s 0.2 --cpu-seconds 0 --no-build $T"
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum -d $out/${v}_tlb -o run -f csv -- python3 $B > $out/${v}_tlb.log 2>&1 || exit $?
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d $out/${v}_tcc -o run -f csv -- python3 $B > $out/${v}_tcc.log 2>&1 || exit $?
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $out/${v}_sq -o run -f csv -- python3 $B > $out/${v}_sq.log 2>&1 || exit $?
done
echo done
