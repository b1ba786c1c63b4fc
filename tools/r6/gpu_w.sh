#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/w
python - <<'PY' > gpurun_out/r6/w/probe.log 2>&1
import os, random, subprocess
os.makedirs('gpurun_out/r6/w/dump', exist_ok=True)
os.makedirs('gpurun_out/r6/w/dump', exist_ok=True)
for (n, nb, p, q, o, poison, trim) in [(1100, 32, 2, 1, 0, '0', 'x'), (1100, 32, 2, 2, 0, '0', 'x'), (700, 32, 2, 1, 0, '0', 'x')]:
    port = random.randint(20000, 50000)
    env = {k: v for k, v in os.environ.items() if not k.startswith("PYTHON")}
    env["LD_LIBRARY_PATH"] = "/opt/rocm/lib"
    ps = []
    for r in range(p * q):
        e = dict(env, RANK=str(r), WORLD_SIZE=str(p * q), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                 MASTER_PORT=str(port), SLATE_AMD_NATIVE_TRANSPORT="host",
                 SLATE_AMD_HEEV_GRID_STOP=poison, SLATE_AMD_NATIVE_HEEV_DUMP="gpurun_out/r6/w/dump")
        ps.append(subprocess.Popen(["tools/r6/heev_probe", str(n), str(nb), str(p), str(q), str(o)], env=e,
                                   stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    for pr in ps:
        out = pr.communicate(timeout=300)[0]
        if out.strip():
            print("STOP", poison, trim, f"{p}x{q}", out, flush=True)
PY
rc=$?
tail -60 gpurun_out/r6/w/probe.log
exit $rc
exit $rc
