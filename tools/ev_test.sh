set -u
for e in 1 10 1000; do
  timeout -k 10 200 python bench.py --steps 400 --cpu-seconds 0 --event-every $e > gpurun_out/ev_$e.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ev_$e.json'));print('every=$e', d['value'], d['ms_per_step'], d['kernel_ms_mean'])"
done
