#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/ag
python - <<'PY' > gpurun_out/r6/ag/probe.log 2>&1
import os, random, subprocess
for (n, nb, p, q, o) in ((1100, 32, 2, 2, 3), (1100, 48, 2, 1, 3), (700, 32, 1, 4, 3)):
    port = random.randint(20000, 50000)
    env = {k: v for k, v in os.environ.items() if not k.startswith("PYTHON")}
    env["LD_LIBRARY_PATH"] = "/opt/rocm/lib"
    ps = []
    for r in range(p * q):
        e = dict(env, RANK=str(r), WORLD_SIZE=str(p * q), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                 MASTER_PORT=str(port), SLATE_AMD_NATIVE_TRANSPORT="host")
        ps.append(subprocess.Popen(["tools/r6/heev_probe", str(n), str(nb), str(p), str(q), str(o)], env=e,
                                   stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    for pr in ps:
        out = pr.communicate(timeout=300)[0]
        if out.strip():
            print(f"{p}x{q} n={n}:", out, flush=True)
PY
rc=$?
grep -v "bad column" gpurun_out/r6/ag/probe.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_native_gpu.py -k "example" > gpurun_out/r6/ag/native.log 2>&1
rc=$?
tail -2 gpurun_out/r6/ag/native.log
exit $rc
