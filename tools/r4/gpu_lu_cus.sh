#!/bin/bash
# dgetrf n = 32768: CUs reserved for the LU panel (32 = default)
for c in 32 48 64 40 32; do
  SLATE_AMD_PANEL_CUS=$c timeout -k 10 120 python bench.py --routine getrf --steps 2 --warmup 1 > /tmp/lu_$c.log 2>&1 || exit $?
  echo "cus=$c $(grep -o '"value": [0-9.]*' /tmp/lu_$c.log)"
done
