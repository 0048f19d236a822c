#!/bin/bash
# Round 3 (session 2): SQ counters of the LDS-form workloads (ragged 15 against receive 13): instruction mix and
# wait cycles per launch (tools/profile.sh groups sq, sq2; one --pmc pass each).
set -u
for c in ${1:-15 13}; do
  GROUPS_ONLY="sq sq2" bash tools/profile.sh $c r03sq || exit 1
done
echo done
