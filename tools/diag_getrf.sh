#!/bin/bash
# getrf backward error across sizes / lookahead (one GPU)
set -o pipefail
mkdir -p gpurun_out
for cfg in "4096 512 1" "4096 512 2" "8192 512 1" "16384 512 0" "32768 512 2"; do
  set -- $cfg
  echo "n=$1 nb=$2 la=$3" >> gpurun_out/diag.log
  timeout -k 10 120 python -u bench.py --routine getrf --n $1 --nb $2 --lookahead $3 --steps 1 --warmup 1 >> gpurun_out/diag.log 2>&1 || exit 1
done
