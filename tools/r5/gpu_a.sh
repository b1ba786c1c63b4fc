#!/bin/bash
# round 5 / a: fp64 MFMA ceiling, same-device IPC probe, stream + native tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5; mkdir -p $D
timeout -k 10 120 ./tools/exp/mfma_peak.bin > $D/mfma_peak2.txt 2>&1 || { cat $D/mfma_peak2.txt; exit 1; }
cat $D/mfma_peak2.txt
for kind in 0 1; do
  T=$(mktemp -d)
  timeout -k 5 40 ./tools/probe/ipc_probe.bin 0 $T $kind > $D/ipc_e$kind.txt 2>&1 &
  E=$!
  timeout -k 5 40 ./tools/probe/ipc_probe.bin 1 $T $kind > $D/ipc_i$kind.txt 2>&1
  ri=$?
  wait $E; re=$?
  echo "ipc kind $kind: exporter rc=$re importer rc=$ri"; cat $D/ipc_e$kind.txt $D/ipc_i$kind.txt
  [ $re -ge 124 ] || [ $ri -ge 124 ] && exit 1
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_nosync_gpu.py tests/test_native_gpu.py > $D/pytest_a.log 2>&1
rc=$?; tail -25 $D/pytest_a.log; exit $rc
