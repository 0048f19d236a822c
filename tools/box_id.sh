set -u
mkdir -p gpurun_out
(rocm-smi --showmemorypartition --showcomputepartition --showclocks 2>&1; rocminfo 2>&1 | grep -E "Marketing|Compute Unit|Uuid" | head -8) > gpurun_out/boxid.txt
grep -E "partition|Partition|mclk|fclk|sclk|Uuid" gpurun_out/boxid.txt | head -20
timeout -k 10 300 python tools/alloc_study.py --config 7 --buffers 2 --variants "xcd_chunk=0;xcd_chunk=99" > gpurun_out/as7c.log 2>&1 && grep SUMMARY gpurun_out/as7c.log
timeout -k 10 300 python tools/alloc_study.py --config 2 --buffers 2 --variants "xcd_chunk=0;xcd_chunk=99" > gpurun_out/as2c.log 2>&1 && grep SUMMARY gpurun_out/as2c.log
