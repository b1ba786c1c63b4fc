#!/bin/bash
# wave-uniform wave index in every kernel: full GPU suite, potrf_mc phases, benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3e/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3e/pytest_gpu.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 120 python -u tools/probe/potrf_mc_phases.py 512 | tail -14 || exit 1
timeout -k 10 120 python -u tools/probe/potrf_tile_lat.py 512 || exit 1
for r in potrf getrf geqrf gemm heev; do
  extra="--steps 5 --warmup 2"
  [ $r = getrf ] && extra="--lookahead 2 --steps 3 --warmup 1"
  [ $r = geqrf ] && extra="--rows 65536 --size 8192 --nb 256 --steps 3 --warmup 1"
  [ $r = gemm ] && extra="--steps 2 --warmup 1"
  [ $r = heev ] && extra="--size 16384 --nb 256 --steps 1 --warmup 1"
  timeout -k 10 300 python -u bench.py --routine $r $extra > gpurun_out/r3e/bench_$r.log 2>&1 || { echo $r failed; tail gpurun_out/r3e/bench_$r.log; exit 1; }
  echo "$r: $(tail -1 gpurun_out/r3e/bench_$r.log | cut -c1-220)"
done
