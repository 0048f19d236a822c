#!/bin/bash
# Same-box A/B of two library builds, for changes a tune field cannot switch: the working tree's library
# against one built from a git ref, in alternating processes (tools/ab.py per workload, default launch shape).
#
#   bash tools/lib_ab.sh build [ref]          # here (CPU): builds <ref> (default HEAD) into network-stack_amd/lib_base/libnsx_csum.so
#   bash tools/lib_ab.sh run "10 11" [pairs]  # on the GPU box: new, base, new, base, ... for each workload
#   AB_EXTRA="--set hi=256" bash tools/lib_ab.sh run 15   # extra tools/ab.py arguments (a workload variant)
#   AB_LIBS="new base x" bash tools/lib_ab.sh run 10       # more builds: x = network-stack_amd/lib_x/libnsx_csum.so
#   AB_PREFIX=verify bash tools/lib_ab.sh run 15            # variant names prefixed (tools/ab.py: verify* = batch verify)
#
# Both builds share include/ and the ABI of the working tree; only use it for kernel-internal changes.
set -eu
cd "$(dirname "$0")/.."
case "${1:-}" in
  build)
    ref=${2:-HEAD}
    tmp=$(mktemp -d)
    git archive "$ref" include network-stack_amd | tar -x -C "$tmp"
    make -s -C "$tmp/network-stack_amd" -j8 lib/libnsx_csum.so
    mkdir -p network-stack_amd/lib_base
    cp "$tmp/network-stack_amd/lib/libnsx_csum.so" network-stack_amd/lib_base/libnsx_csum.so
    rm -rf "$tmp"
    echo "network-stack_amd/lib_base/libnsx_csum.so built from $(git rev-parse --short "$ref")"
    ;;
  run)
    configs=${2:-2}
    pairs=${3:-2}
    lib=network-stack_amd/lib/libnsx_csum.so
    cp "$lib" /tmp/lib_ab_new.so
    trap 'cp /tmp/lib_ab_new.so "$lib"' EXIT
    for ((i = 0; i < pairs; i++)); do
      for k in ${AB_LIBS:-new base}; do
        if [ "$k" = new ]; then cp /tmp/lib_ab_new.so "$lib"; else cp "network-stack_amd/lib_$k/libnsx_csum.so" "$lib"; fi
        for c in $configs; do
          timeout -k 10 200 python tools/ab.py --config "$c" --variants "${AB_PREFIX:-}$k:" --rounds 5 ${AB_EXTRA:-} 2>/dev/null | grep AB
        done
      done
    done
    ;;
  *)
    echo "usage: $0 build [ref] | run \"configs\" [pairs]" >&2
    exit 2
    ;;
esac
