#!/bin/bash
# sha256 of the product gfx950 code object built from a csum_kernels.hip (default: the working tree's; or a git
# revision's with REV=<rev>), with a fixed -cuid so that two builds of the same source are byte-identical. Used to
# show that a source change is code-neutral (e.g. the WaveStamps hook).
#   bash tools/codeobj_hash.sh            # working tree
#   REV=HEAD bash tools/codeobj_hash.sh   # a revision
set -eu
cd "$(dirname "$0")/.."
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
src=network-stack_amd/csrc/csum_kernels.hip
if [ -n "${REV:-}" ]; then git show "$REV:$src" > "$tmp/k.hip"; cp network-stack_amd/csrc/csum_kernels.h "$tmp/"; src=$tmp/k.hip; fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I"$PWD/include" -I"$PWD/network-stack_amd/csrc" --offload-arch=gfx950 \
    -munsafe-fp-atomics -cuid=nsx --cuda-device-only -c "$src" -o "$tmp/d.o"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$tmp/d.o" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$tmp/d.co"
sha256sum "$tmp/d.co" | cut -d' ' -f1
