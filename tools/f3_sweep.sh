set -u
for k in 0 1; do for b in 1 2 4 8; do
  timeout -k 10 200 python bench.py --config 7 --steps 100 --cpu-seconds 0 --param kernel=$k --param blocks_per_cu=$b > gpurun_out/c7_k${k}_b$b.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c7_k${k}_b$b.json'));print('kernel=$k bpc=$b', d['kernel_ms_mean'], d['roofline']['frac'])"
done; done
