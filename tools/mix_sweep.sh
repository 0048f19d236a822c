# Receive pass and ragged checksum over other traffic mixes (tools/ab.py --set lo=.. --set hi=..)
set -e
ab() { timeout -k 10 200 python tools/ab.py "$@" --rounds 5 2>&1 | grep AB; }
ab --config 10 --n 8388608 --set lo=40 --set hi=100 --variants "rx:;scan:"
ab --config 10 --n 4194304 --set lo=40 --set hi=300 --variants "rx:;scan:"
ab --config 10 --n 1048576 --set lo=1500 --set hi=1500 --variants "rx:;scan:"
ab --config 3 --n 8388608 --set lo=64 --set hi=256 --variants "def:"
ab --config 3 --n 4194304 --set lo=64 --set hi=1500 --variants "def:"
