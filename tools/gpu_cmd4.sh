set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/drift.py --config 2 --launches 600 > gpurun_out/drift_c2.log 2>&1 || exit 1
cat gpurun_out/drift_c2.log | grep rep
timeout -k 10 300 python tools/drift.py --config 4 --launches 200 > gpurun_out/drift_c4.log 2>&1 || exit 1
cat gpurun_out/drift_c4.log | grep rep
