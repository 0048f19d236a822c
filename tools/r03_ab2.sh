#!/bin/bash
# Round 3 pass 3: parity of the LDS forms (receive pass + ragged), their A/B on the small-frame workloads and
# around the crossover, the TCP build's occupancy A/B, then counters on the LDS form.
set -u
out=gpurun_out/${1:-r03c}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_zz_fuzz.py tests/test_gpu_parity.py \
    tests/test_gpu_00_baseline.py -k "rx or ragged or config3" -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/pytest_rx.log" 2>&1
rc=$?; tail -3 "$out/pytest_rx.log"; [ $rc -eq 0 ] || exit $rc
ab() {  # ab <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > "$out/ab_$tag.txt" 2>&1
  local rc=$?; echo "== $tag rc=$rc"; tail -5 "$out/ab_$tag.txt" | cut -c1-150; [ $rc -eq 0 ] || exit $rc
}
V="auto:;lds:segs_per_wave=2;s4:segs_per_wave=4;s1:segs_per_wave=1"
ab c13 --config 13 --variants "$V" --rounds 5
ab c16 --config 16 --variants "$V" --rounds 5
ab c15 --config 15 --variants "$V" --rounds 5
for hi in 160 220 300; do
  ab c13_hi$hi --config 13 --set hi=$hi --n $((560000000 / (20 + hi))) --variants "$V" --rounds 5
done
for hi in 256 384 512; do
  ab c15_hi$hi --config 15 --set hi=$hi --n $((700000000 / (32 + hi / 2))) --variants "$V" --rounds 5
done
ab c10 --config 10 --variants "$V" --rounds 5
ab c3 --config 3 --variants "$V" --rounds 5
ab c6 --config 6 --variants "def:;b3:blocks_per_cu=3;b4:blocks_per_cu=4;b3g8:blocks_per_cu=3,run_segs=8;b4g8:blocks_per_cu=4,run_segs=8" --rounds 5
ab c8 --config 8 --variants "def:;b3:blocks_per_cu=3;b4:blocks_per_cu=4" --rounds 5
B="bench.py --config 13 --steps 50 --warmup 5 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT -d "$out/pmc13a" -o run -f csv \
    -- python3 $B > "$out/pmc13a.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d "$out/pmc13b" -o run -f csv \
    -- python3 $B > "$out/pmc13b.log" 2>&1 || exit $?
echo done
