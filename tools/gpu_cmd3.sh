set -u
mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
for c in 2 3 4; do timeout -k 10 300 python bench.py --config $c --steps 100 --cpu-seconds 0 > gpurun_out/bench_c$c.log 2>&1 || exit 1; tail -1 gpurun_out/bench_c$c.log | cut -c1-400; done
bash tools/profile.sh 2 r01
