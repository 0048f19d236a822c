set -u
mkdir -p gpurun_out
timeout -k 10 600 python tools/shape_sweep.py --shapes 1500:1500,2048:2048,3000:3000,8192:8192,65536:65536 --param "xcd_map=3" --param "xcd_map=3;blocks_per_cu=2" --param "xcd_map=3;blocks_per_cu=8" --param "xcd_map=3;segs_per_wave=2" --param "xcd_map=3;segs_per_wave=1;blocks_per_cu=8" --param "xcd_map=2" > gpurun_out/shape2.log 2>&1; echo rc=$?
grep L= gpurun_out/shape2.log
timeout -k 10 600 python tools/sweep.py --configs 3,2 --rounds 3 --iters 10 > gpurun_out/sweep2.log 2>&1; echo rc=$?
grep -v round gpurun_out/sweep2.log | grep config | cut -c1-200
