#!/bin/bash
# rocprofv3 evidence for one bench workload: kernel-trace stats, then each PMC
# group in its own pass (never combined with other trace domains).
# usage: [GROUPS_ONLY="kt fetch write sq sq2 icache lds tlb tcc"] [BENCH_EXTRA="--no-pseudo"] tools/profile.sh <config> [tag] [label]
# (label names the output directory, default the config number: e.g. 2n for config 2 with --no-pseudo)
set -u
cfg=${1:-2}; tag=${2:-r01}; label=${3:-$cfg}
out=gpurun_out/prof_${tag}_c${label}
mkdir -p "$out"
export TMPDIR=/tmp
# the library is built here, before rocprofv3 starts (its preloaded library initialises the GPU first), and bench.py
# loads it as it is (--no-build): no compiler runs as a child of a profiled process
[ -n "${NO_MAKE:-}" ] || make -s -j16 -C network-stack_amd || exit 1  # NO_MAKE: a library swapped in by tools/valu_ab.sh
B="bench.py --config $cfg --steps 50 --warmup 5 --cpu-seconds 0 --no-build ${BENCH_EXTRA:-}"
run() {  # run <name> <timeout> rocprofv3-args...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" rocprofv3 "$@" -d "$out/$name" -o run -f csv -- python3 $B > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$out/$name.log" | cut -c1-200
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc"; exit $rc; fi
}
want() { [ -z "${GROUPS_ONLY:-}" ] || [[ " $GROUPS_ONLY " == *" $1 "* ]]; }
if want kt; then run kt 300 --kernel-trace --stats; fi
if want fetch; then run fetch 300 --kernel-trace --pmc FETCH_SIZE; fi
if want write; then run write 300 --kernel-trace --pmc WRITE_SIZE; fi
if want sq; then run sq 300 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE; fi
if want sq2; then run sq2 300 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR; fi
if want tlb; then run tlb 300 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum; fi
if want icache; then run icache 300 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE; fi
if want lds; then run lds 300 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_IDX_ACTIVE; fi
if want tcc; then run tcc 300 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum; fi
