# Receive pass: runs of 1 / 4 frame sets and the automatic choice over frame mixes (tools/ab.py --set)
set -e
for m in "40 100 8388608" "40 160 6291456" "40 220 4194304" "40 300 4194304" "40 1500 1048576"; do
  set -- $m
  timeout -k 10 200 python tools/ab.py --config 10 --n $3 --set lo=$1 --set hi=$2 --variants "auto:;s1:segs_per_wave=1;s4:segs_per_wave=4" --rounds 5 2>&1 | grep AB
done
