#!/bin/bash
# 1-GPU native heev n=16384: per-stage spans from the native trace
set -o pipefail
mkdir -p gpurun_out/r6/x
SLATE_AMD_NATIVE_TRACE=$PWD/gpurun_out/r6/x/heev16k_trace.json timeout -k 10 300 slate_amd/bench_native heev 16384 256 1 1 1 1 1 0 > gpurun_out/r6/x/heev16k.log 2>&1
rc=$?
cat gpurun_out/r6/x/heev16k.log
[ $rc -ne 0 ] && exit $rc
python - <<'PY' | tee gpurun_out/r6/x/heev16k_stages.txt
import json, collections
ev = json.load(open("gpurun_out/r6/x/heev16k_trace.json"))["traceEvents"]
tot = collections.defaultdict(float)
for e in ev:
    if e.get("ph") == "X":
        tot[(e["name"], e["tid"])] += e["dur"] / 1e3
for (nm, tid), ms in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"{nm:32s} track {tid}: {ms:10.1f} ms")
PY
