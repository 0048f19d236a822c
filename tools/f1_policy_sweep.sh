set -u
for p in 1 2 3 4; do
  timeout -k 10 200 python bench.py --config 6 --steps 100 --cpu-seconds 0 --param nontemporal=$p > gpurun_out/c6_p$p.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c6_p$p.json'));print($p, d['kernel_ms_mean'], d['roofline']['frac'])"
done
