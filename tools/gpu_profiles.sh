#!/bin/bash
# GPU evidence pass, part 2: rocprofv3 kernel stats + PMC traffic per workload,
# summarised into profiles/ by tools/prof_summary.py.
set -u
tag=${1:-r02}
for c in ${PROFILE_CONFIGS:-2 3 4 5 6 7 8 9 10}; do
  bash tools/profile.sh $c $tag || exit 1
  python3 tools/prof_summary.py $tag $c > /dev/null || exit 1
  echo "profiled config $c"
done
