set -u
mkdir -p gpurun_out
timeout -k 10 600 python tools/shape_sweep.py --param "segs_per_wave=1;blocks_per_cu=8" --param "segs_per_wave=2;blocks_per_cu=8" --param "kernel=1" --param "kernel=1;blocks_per_cu=2;stream_rows=4" --param "blocks_per_cu=2" --param "blocks_per_cu=8" > gpurun_out/shape.log 2>&1; echo rc=$?
cat gpurun_out/shape.log | grep -v amdgpu.ids
