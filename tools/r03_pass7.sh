#!/bin/bash
# Round 3 pass 7: the LDS forms without byte masks (lds_range_sum's head from the chunk's dword prefix sums and
# tail from the next lane by DPP; header sums from rotated frame-relative dwords): small-frame parity first, then
# a same-box A/B against the HEAD build (tools/lib_ab.sh), then the TCP build's ds_bpermute variant A/B + SQ
# counters, then the whole -m gpu suite.
set -u
out=gpurun_out/${1:-r03i}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "small or ragged or rx" > "$out/pytest_focus.log" 2>&1
rc=$?; tail -2 "$out/pytest_focus.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/lib_ab.sh run "13 15 16 14 10 3" 2 > "$out/lib_ab.txt" 2>&1 || exit $?
cat "$out/lib_ab.txt"
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
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$out/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo done
