#!/bin/bash
# Round-3 profiling evidence: heev kernel table (n=16384), PMC passes
# (potrf / getrf n=16384, heev n=8192), dgemm n=32768 bench line.
# Each step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3g
mkdir -p $O
C="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"
timeout -k 10 240 python -u bench.py --routine gemm --n 32768 --steps 3 --warmup 1 > $O/bench_gemm32k.log 2>&1 &&
tail -1 $O/bench_gemm32k.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/heev -o heev -- python3 bench.py --routine heev --n 16384 --nb 256 --steps 1 --warmup 1 --check 0 > $O/heev.log 2>&1 &&
tail -2 $O/heev.log &&
timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $O/pmc_potrf -o potrf -- python3 bench.py --routine potrf --n 16384 --steps 1 --warmup 0 --check 0 > $O/pmc_potrf.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $O/pmc_getrf -o getrf -- python3 bench.py --routine getrf --n 16384 --lookahead 2 --steps 1 --warmup 0 --check 0 > $O/pmc_getrf.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/pmc_heev -o heev -- python3 bench.py --routine heev --n 8192 --nb 256 --steps 1 --warmup 0 --check 0 > $O/pmc_heev.log 2>&1
rc=$?
echo "chain rc=$rc"
for w in potrf getrf heev; do [ -d $O/pmc_$w ] && python3 tools/pmc_summary.py $O/pmc_$w 10 > $O/pmc_$w.txt 2>&1; done
db=$(find $O/heev -name "*.db" | head -1); [ -n "$db" ] && python3 tools/prof_summary.py "$db" 30 > $O/heev_kernels.txt 2>&1
find $O -name "*.db" -size +60M -delete
find $O -name "*.csv" -size +40M -delete
exit $rc
