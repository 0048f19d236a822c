# Ragged checksum: runs of four 63-segment sets for small segments. Same-process mixes (auto / forced two sets via
# segs_per_wave=2 is not a knob: s4 forces four), then config 3 against the base library (tools/lib_ab.sh).
set -e
ab() { timeout -k 10 200 python tools/ab.py "$@" --rounds 5 2>&1 | grep AB; }
for m in "64 128 8388608" "64 192 8388608" "64 256 8388608" "64 1500 4194304"; do
  set -- $m
  ab --config 3 --n $3 --set lo=$1 --set hi=$2 --variants "auto:;s4:segs_per_wave=4;s1:segs_per_wave=1"
done
bash tools/lib_ab.sh run "3" 2
