"""Run every example (reference examples/run_tests.py); exits non-zero on failure.
    python examples/run_examples.py            # single process
    python examples/run_examples.py --np 2     # torchrun with 2 ranks (gloo on CPU)"""
import argparse
import glob
import os
import subprocess
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--np", type=int, default=1)
a = ap.parse_args()
here = os.path.dirname(os.path.abspath(__file__))
root = os.path.dirname(here)
env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
fails = 0
for ex in sorted(glob.glob(os.path.join(here, "ex*.py"))):
    cmd = [sys.executable, ex] if a.np == 1 else \
        [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(a.np),
         "--master-addr", "127.0.0.1", "--master-port", "29611", ex]
    r = subprocess.run(cmd, env=env, cwd=root, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=600)
    ok = r.returncode == 0
    fails += not ok
    print(("pass " if ok else "FAIL ") + os.path.basename(ex))
    if not ok:
        print(r.stdout[-3000:])
sys.exit(1 if fails else 0)
