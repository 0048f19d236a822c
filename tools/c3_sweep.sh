mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 200 python bench.py --config 3 --steps 100 --cpu-seconds 0 "$@" > gpurun_out/c3_$tag.log 2>&1 || exit 1; python -c "import json; d=json.loads(open('gpurun_out/c3_$tag.log').read().splitlines()[-1]); print('$tag', d['kernel_ms_mean'], d['roofline']['frac'])"; }
for r in 1 2; do
run def
run b1k6 --param blocks_per_cu=1 --param kernel=6
run b1k6r16 --param blocks_per_cu=1 --param kernel=6 --param stream_rows=16
run b1r16 --param blocks_per_cu=1 --param stream_rows=16
run b3 --param blocks_per_cu=3
run r16 --param stream_rows=16
done
