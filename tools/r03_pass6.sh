#!/bin/bash
# Round 3 pass 6: the whole -m gpu suite on the current tree, then the TCP build's ds_bpermute header variant
#  against the default in one process, with SQ instruction counters for both.
set -u
out=gpurun_out/${1:-r03h}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$out/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
for c in 6 8; do
  timeout -k 10 300 python -u tools/ab.py --config $c --variants "def:;bperm:kernel=4" --rounds 7 > "$out/ab_c$c.txt" 2>&1 || exit $?
  grep "^AB" "$out/ab_c$c.txt"
done
for v in "" "--tune kernel=4"; do
  tag=$([ -z "$v" ] && echo def || echo bperm)
  B="bench.py --config 6 --steps 50 --warmup 5 --cpu-seconds 0 $v"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR -d "$out/pmc6_$tag" -o run -f csv \
      -- python3 $B > "$out/pmc6_$tag.log" 2>&1 || exit $?
done
echo done
