#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3d
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_qr.py tests/test_nosync_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "potrf or cholqr or geqrf" > gpurun_out/r3d/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r3d/pytest.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 120 python -u tools/probe/potrf_mc_phases.py 512 || exit 1
for n in 512 256; do timeout -k 10 120 python -u tools/probe/potrf_tile_lat.py $n || exit 1; done
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r3d/bench_potrf.log 2>&1 || { echo potrf failed; tail gpurun_out/r3d/bench_potrf.log; exit 1; }
echo "potrf: $(tail -1 gpurun_out/r3d/bench_potrf.log | cut -c1-200)"
timeout -k 10 200 python -u bench.py --routine geqrf --rows 65536 --size 8192 --nb 256 --steps 3 --warmup 1 > gpurun_out/r3d/bench_geqrf.log 2>&1 || { echo geqrf failed; tail gpurun_out/r3d/bench_geqrf.log; exit 1; }
echo "geqrf: $(tail -1 gpurun_out/r3d/bench_geqrf.log | cut -c1-200)"
