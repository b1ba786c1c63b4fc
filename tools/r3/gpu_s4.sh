#!/bin/bash
# LU base: DPP arg-max + single-barrier publish; hb2st lag 3; unmtr_hb2st Y = V T (two GEMMs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-s4}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py tests/test_nosync_gpu.py tests/test_eig_svd.py -m gpu -x -q --timeout 120 --timeout-method thread -k "getrf or lu or gesv or hb2st or heev or unmtr or trsm" > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u tools/probe/lu_panel_time.py > $D/lu_panel_time.log 2>&1 || { tail $D/lu_panel_time.log; exit 1; }
cat $D/lu_panel_time.log
timeout -k 10 200 python -u bench.py --routine getrf --lookahead 2 --steps 3 --warmup 1 > $D/bench_getrf.log 2>&1 || { tail $D/bench_getrf.log; exit 1; }
tail -1 $D/bench_getrf.log
HB2ST_PROBE_NOHOST=1 timeout -k 10 200 python -u tools/probe/hb2st_time.py 16384 64 > $D/hb2st.log 2>&1 || { tail $D/hb2st.log; exit 1; }
cat $D/hb2st.log
timeout -k 10 300 python -u bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 1 > $D/bench_heev.log 2>&1 || { tail $D/bench_heev.log; exit 1; }
tail -1 $D/bench_heev.log
