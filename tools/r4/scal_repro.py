import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from tests.test_native_gpu import _run_ranks, ROOT
exe = os.path.join(ROOT, "slate_amd", "scal_probe")
variants = [("2x1", "0", {}), ("2x2", "0", {}), ("1x2", "0", {})]
for it in range(int(sys.argv[1])):
    for grid, warm, v in variants:
        p, q = map(int, grid.split("x"))
        outs = _run_ranks(exe, [grid, "384", "32", warm], p * q, timeout=120)
        first = [l for l in outs[0][1].splitlines() if l.startswith("rep 0")]
        print(f"iter {it} {grid} warm={warm} {v} rc={[o[0] for o in outs]} {first}", flush=True)
