set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 600 python tools/sweep.py --configs 3 --rounds 3 --iters 10 > gpurun_out/sweep4.log 2>&1; echo "sweep rc=$?"
grep -v round gpurun_out/sweep4.log | grep config | cut -c1-200
