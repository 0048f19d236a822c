set -u
timeout -k 10 300 python tools/drift.py --config 2 --launches 2000 > gpurun_out/drift2.log 2>&1; echo rc=$?
grep rep gpurun_out/drift2.log
