set -u
for c in 3 4; do bash tools/profile.sh $c r01 || exit 1; done
