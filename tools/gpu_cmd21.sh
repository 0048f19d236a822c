set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x -k "tcp_build or ipv4" > gpurun_out/pytest_new.log 2>&1; echo "pytest rc=$?"; tail -30 gpurun_out/pytest_new.log | grep -v Warning
