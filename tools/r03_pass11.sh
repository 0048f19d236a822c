#!/bin/bash
# Round 3 pass 11 = pass 10 (4-chunk follow-up blocks: parity + A/B against HEAD) then the count-range experiment.
set -u
bash tools/r03_pass10.sh ${1:-r03l} || exit $?
bash tools/r03_exp_ranges.sh ${2:-r03m} || exit $?
