#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_eig_svd.py -x -v --timeout 150 --timeout-method thread -m gpu > gpurun_out/pytest_eig.log 2>&1 || { tail -40 gpurun_out/pytest_eig.log; exit 1; }
tail -2 gpurun_out/pytest_eig.log
for band in 64; do
  SLATE_AMD_HB2ST=device timeout -k 10 300 python -u tools/heev_phases.py 16384 256 $band > gpurun_out/heev_phases_$band.log 2>&1 || { cat gpurun_out/heev_phases_$band.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/heev_phases_$band.log | grep -v "  host"
done
mkdir -p gpurun_out/pc_heev2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc_heev2 -o heev -- python3 tools/heev_phases.py 16384 256 > gpurun_out/pc_heev2/run.log 2>&1
find gpurun_out/pc_heev2 -name "*kernel_trace.csv" -size +50M -delete
python3 tools/prof_csv_summary.py gpurun_out/pc_heev2 14 || true
timeout -k 10 240 python -u bench.py --routine getrf --method calu --lookahead 2 --steps 2 --warmup 1 > gpurun_out/bench_getrf_calu.log 2>&1 || { tail -20 gpurun_out/bench_getrf_calu.log; exit 1; }
grep -h '"metric"' gpurun_out/bench_getrf_calu.log
