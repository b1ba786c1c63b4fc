"""Repeat the 2x2 host-transport native runs to catch an intermittent error."""
import os, sys, subprocess
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from tests.test_native_gpu import _run_ranks, EXE, CEXE
os.environ["EX_NATIVE_TYPES"] = "d"
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    for n, nb in ((384, 32), (300, 32)):
        os.environ["EX_NATIVE_N"], os.environ["EX_NATIVE_NB"] = str(n), str(nb)
        outs = _run_ranks(EXE, ["2x2"], 4, timeout=120)
        bad = [l for l in outs[0][1].splitlines() if l.startswith("check") and float(l.split()[2]) > 1e-12]
        print(f"iter {it} ex_native n={n} rc={[o[0] for o in outs]} bad={bad}", flush=True)
    outs = _run_ranks(CEXE, ["2x2"], 4, timeout=120)
    bad = [l for rc, o in outs for l in o.splitlines() if l.startswith("check") and float(l.split()[3]) > 1e-11]
    print(f"iter {it} scalapack rc={[o[0] for o in outs]} bad={bad}", flush=True)
