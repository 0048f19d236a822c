set -u
for i in 1 2; do timeout -k 10 300 python bench.py --cpu-seconds 2 > gpurun_out/bench_rep$i.log 2>&1 || exit 1; tail -1 gpurun_out/bench_rep$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms_mean'], d['roofline']['frac'])"; done
timeout -k 10 300 python bench.py --cpu-seconds 0 --settle-s 2 > gpurun_out/bench_rep3.log 2>&1 || exit 1; tail -1 gpurun_out/bench_rep3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('settle2', d['value'], d['kernel_ms_mean'], d['roofline']['frac'])"
