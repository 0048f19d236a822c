#!/bin/bash
# Experiment: count-based wave ranges (no offsets search) for the receive / ragged kernels, built into
# network-stack_amd/lib_exp (not a product path): FETCH_SIZE and time against the working tree's library.
set -u
out=gpurun_out/${1:-r03m}
mkdir -p "$out"
export TMPDIR=/tmp
lib=network-stack_amd/lib/libnsx_csum.so
cp "$lib" /tmp/lib_new.so
trap 'cp /tmp/lib_new.so "$lib"' EXIT
for k in new exp new exp; do
  if [ "$k" = exp ]; then cp network-stack_amd/lib_exp/libnsx_csum.so "$lib"; else cp /tmp/lib_new.so "$lib"; fi
  for c in 13 15 10 14; do
    timeout -k 10 200 python tools/ab.py --config $c --variants "$k:" --rounds 5 2>/dev/null | grep AB
  done
done
for k in new exp; do
  if [ "$k" = exp ]; then cp network-stack_amd/lib_exp/libnsx_csum.so "$lib"; else cp /tmp/lib_new.so "$lib"; fi
  for c in 13 15; do
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$out/f_${k}_$c" -o run -f csv \
      -- python3 bench.py --config $c --steps 20 --warmup 5 --cpu-seconds 0 > "$out/f_${k}_$c.log" 2>&1 || exit $?
    python3 - "$out/f_${k}_$c/run_counter_collection.csv" $k $c <<'PY'
import csv, sys, statistics
rows = [r for r in csv.DictReader(open(sys.argv[1])) if ("rx_tcp" in r["Kernel_Name"] or "ragged_scan" in r["Kernel_Name"])]
v = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == "FETCH_SIZE"]
print("FETCH", sys.argv[2], "config", sys.argv[3], "launches", len(v), "bytes/launch x2 corrected", statistics.mean(v) * 2048)
PY
  done
done
echo done
