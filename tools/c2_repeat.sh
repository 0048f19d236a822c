#!/bin/bash
# Config-2 bench repeated in fresh processes on one box (box warm-up / settle-time study).
# usage: bash tools/c2_repeat.sh "<settle seconds per run>"   e.g. "3 0.5 3"
set -u
mkdir -p gpurun_out
i=0
for s in ${1:-0.5 0.5 0.5}; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --cpu-seconds 0 --settle-s $s > gpurun_out/c2rep_$i.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/c2rep_$i.log').read().strip().splitlines()[-1]);print('rep $i settle $s', d['value'], d['kernel_ms_mean'], d['roofline']['frac'])"
done
