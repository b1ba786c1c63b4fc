#!/bin/bash
# full GPU suite on the current tree; heev band sweep (stage-1 band 64 / 32 / 48)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s8}; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest.log
[ $rc -ne 0 ] && exit 1
for b in 64 32 48; do
  timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --band $b --steps 2 --warmup 1 > $D/bench_heev_$b.log 2>&1 || { tail $D/bench_heev_$b.log; exit 1; }
  echo "band $b: $(tail -1 $D/bench_heev_$b.log | cut -c1-120)"
done
