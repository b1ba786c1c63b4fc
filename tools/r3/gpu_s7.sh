#!/bin/bash
# wide split-K fp64 GEMM + tri_inv op tests; dgetrf explicit-inverse U rows sweep; heev kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s7}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_eig_svd.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or trsm or heev or unmtr or hb2st" > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest.log
[ $rc -ne 0 ] && exit 1
for v in 0 2048 8192; do
  SLATE_AMD_LU_INV_MIN=$v timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/bench_getrf_$v.log 2>&1 || { tail $D/bench_getrf_$v.log; exit 1; }
  echo "inv_min $v: $(tail -1 $D/bench_getrf_$v.log | cut -c1-150)"
done
timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --steps 2 --warmup 1 > $D/bench_heev.log 2>&1 || { tail $D/bench_heev.log; exit 1; }
tail -1 $D/bench_heev.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_heev -o run -- python3 $GRAFT_REPO_ROOT/bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 0 > $GRAFT_REPO_ROOT/$D/prof_heev.log 2>&1
echo "prof rc=$?"
