# XCD deal balance A/B (new library vs lib_ab base) at batch sizes that are not powers of two
set -e
lib=network-stack_amd/lib/libnsx_csum.so
cp "$lib" /tmp/new.so
trap 'cp /tmp/new.so "$lib"' EXIT
ab() { timeout -k 10 200 python tools/ab.py "$@" --rounds 5 2>&1 | grep AB; }
for k in new base new base; do
  if [ $k = base ]; then cp lib_ab/libnsx_csum.so "$lib"; else cp /tmp/new.so "$lib"; fi
  echo "== $k"
  ab --config 2 --n 1000000 --variants "$k:"
  ab --config 6 --n 1000000 --variants "$k:"
  ab --config 7 --n 60000000 --variants "$k:;${k}_w3:window_bytes=447392427"
  ab --config 9 --n 60000000 --variants "$k:"
done
