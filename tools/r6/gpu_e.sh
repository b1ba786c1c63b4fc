#!/bin/bash
# round 6 / e: fresh-container rebuild check -- full GPU suite, 1-GPU dpotrf +
# dgetrf bench, PMC row of the glds GEMM (MFMA busy, LDS conflicts, L2 hit)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6/e; mkdir -p $D
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1
rc=$?; tail -4 $D/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > $D/bench_potrf.txt 2>&1
rc=$?; tail -1 $D/bench_potrf.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --routine getrf --steps 5 --warmup 2 > $D/bench_getrf.txt 2>&1
rc=$?; tail -1 $D/bench_getrf.txt; [ $rc -eq 0 ] || exit $rc
C="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"
timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $D/pmc_potrf -o potrf -- python3 bench.py --routine potrf --n 16384 --steps 1 --warmup 0 --check 0 > $D/pmc_potrf.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py $D/pmc_potrf 10 > $D/pmc_potrf.txt 2>&1; cat $D/pmc_potrf.txt
find $D -name "*.csv" -size +50M -delete
exit 0
