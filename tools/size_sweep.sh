set -e
ab() { timeout -k 10 200 python tools/ab.py "$@" --rounds 5 2>&1 | grep AB; }
for n in 524288 1048576 2097152; do ab --config 10 --n $n --variants "b3:;b2:blocks_per_cu=2;b4:blocks_per_cu=4"; done
for n in 262144 524288 1048576 2097152; do ab --config 3 --n $n --variants "def:"; done
for n in 524288 1048576 2097152; do ab --config 2 --n $n --variants "def:"; done
for n in 33554432 67108864 134217728; do ab --config 7 --n $n --variants "def:"; ab --config 9 --n $n --variants "def:"; done
