#!/bin/bash
# Round 3 (session 2): the receive pass ring form (removed after this A/B): receive-pass parity (every form and the
# fuzz), then same-process A/B against the default on the large-frame workloads.
set -u
out=gpurun_out/${1:-r03r}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_zz_fuzz.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "rx" > "$out/pytest.log" 2>&1
rc=$?; tail -3 "$out/pytest.log"; [ $rc -eq 0 ] || exit $rc
V="def:;ring4:segs_per_wave=8;ring3:segs_per_wave=9;p2:segs_per_wave=6"
for c in 10 11 14 18 17; do
  timeout -k 10 200 python tools/ab.py --config $c --variants "$V" --rounds 5 > "$out/ab_c$c.txt" 2>&1 || exit $?
  grep AB "$out/ab_c$c.txt"
done
timeout -k 10 200 python tools/ab.py --config 13 --set hi=1000 --variants "$V" --rounds 5 > "$out/ab_h1000.txt" 2>&1 || exit $?
grep AB "$out/ab_h1000.txt"
echo done
