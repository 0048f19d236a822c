#!/bin/bash
# GPU evidence pass, part 2: rocprofv3 kernel stats + PMC traffic per workload,
# summarised into profiles/ by tools/prof_summary.py. Only gpurun_out/ comes back
# from the GPU box (≤ 64 MiB), so the summaries are copied to gpurun_out/profiles/
# and each config's raw rocprofv3 output is deleted once it is summarised;
# copy gpurun_out/profiles/* into profiles/ afterwards.
set -u
tag=${1:-r02}
mkdir -p gpurun_out/profiles
for c in ${PROFILE_CONFIGS:-2 3 4 5 6 7 8 9 10 11 12}; do
  bash tools/profile.sh $c $tag || exit 1
  python3 tools/prof_summary.py $tag $c > /dev/null || exit 1
  cp profiles/${tag}_config${c}.md profiles/${tag}_config${c}_kernel_stats.csv profiles/traffic_config${c}.json gpurun_out/profiles/ || exit 1
  rm -rf gpurun_out/prof_${tag}_c${c}
  echo "profiled config $c"
done
