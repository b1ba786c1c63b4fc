#!/bin/bash
# potrf_mc: tile tests, tile latency (alone / loaded), dpotrf + dgeqrf benches with each tile kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3b
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "potrf" > gpurun_out/r3b/pytest_potrf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r3b/pytest_potrf.log
[ $rc -ne 0 ] && exit 1
for n in 512 256; do timeout -k 10 120 python -u tools/probe/potrf_tile_lat.py $n || exit 1; done
for v in mc lds; do
  SLATE_AMD_POTRF_TILE=$v timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r3b/bench_potrf_$v.log 2>&1 || { echo potrf $v failed; tail gpurun_out/r3b/bench_potrf_$v.log; exit 1; }
  echo "potrf $v: $(tail -1 gpurun_out/r3b/bench_potrf_$v.log | cut -c1-200)"
  SLATE_AMD_POTRF_TILE=$v timeout -k 10 200 python -u bench.py --routine geqrf --rows 65536 --size 8192 --nb 256 --steps 3 --warmup 1 > gpurun_out/r3b/bench_geqrf_$v.log 2>&1 || { echo geqrf $v failed; tail gpurun_out/r3b/bench_geqrf_$v.log; exit 1; }
  echo "geqrf $v: $(tail -1 gpurun_out/r3b/bench_geqrf_$v.log | cut -c1-200)"
done
