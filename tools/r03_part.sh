#!/bin/bash
# Round 3 (session 2): lds_range_sum's partials loaded one run ahead, none without partials, in the ragged LDS form: parity of the
# LDS forms, then alternating library builds (tools/lib_ab.sh) against HEAD on the LDS-form workloads.
set -u
out=gpurun_out/${1:-r03l4}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_00_baseline.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "ragged" > "$out/pytest.log" 2>&1
rc=$?; tail -3 "$out/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash tools/lib_ab.sh run "15 3" 3 > "$out/lib_ab.txt" 2>&1 || exit $?
cat "$out/lib_ab.txt"
echo done
