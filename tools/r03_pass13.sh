#!/bin/bash
# Round 3 pass 13: receive-pass LDS runs cut to the whole 8-frame groups that fit the slot (instead of streaming
# the whole 64-frame run): receive parity, then alternating library builds against HEAD.
set -u
out=gpurun_out/${1:-r03o}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > "$out/pytest_rx.log" 2>&1
rc=$?; tail -2 "$out/pytest_rx.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash tools/lib_ab.sh run "17 13 16 14 10" 2 > "$out/lib_ab.txt" 2>&1 || exit $?
cat "$out/lib_ab.txt"
for v in "auto:" "s1:segs_per_wave=1" "s2:segs_per_wave=2" "b3:blocks_per_cu=3"; do
  timeout -k 10 200 python tools/ab.py --config 17 --variants "$v" --rounds 5 2>/dev/null | grep AB
done
echo done
