#!/bin/bash
# native p x q getrf rehearsal on one GPU (host transport, 2x1): lookahead 0 vs 1
set -o pipefail
mkdir -p gpurun_out/r6/aj
python - <<'PY' 2>&1 | tee gpurun_out/r6/aj/rehearsal.txt
import os, random, subprocess
for la in (0, 1):
    port = random.randint(20000, 50000)
    env = {k: v for k, v in os.environ.items() if not k.startswith("PYTHON")}
    env["LD_LIBRARY_PATH"] = "/opt/rocm/lib"
    ps = []
    for r in range(2):
        e = dict(env, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                 MASTER_PORT=str(port), SLATE_AMD_NATIVE_TRANSPORT="host")
        ps.append(subprocess.Popen(["slate_amd/bench_native", "getrf", "8192", "512", "2", "1", str(la), "1", "2", "1"],
                                   env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=300)[0] for p in ps]
    print(f"2x1 n=8192 la={la}:", [l for l in outs[0].splitlines() if "RESULT" in l], flush=True)
PY
