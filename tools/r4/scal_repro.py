import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from tests.test_native_gpu import _run_ranks, ROOT
exe = os.path.join(ROOT, "slate_amd", "scal_probe")
variants = [("2x1", w, {}) for w in ("0", "2", "3", "4", "5")]
for it in range(int(sys.argv[1])):
    for grid, warm, v in variants:
        for k in ("SLATE_AMD_NATIVE_SERIAL", "SLATE_AMD_POTRF_CHUNK", "SLATE_AMD_POTRF_TILE", "SLATE_AMD_NATIVE_POISON"):
            os.environ.pop(k, None)
        os.environ.update(v)
        p, q = map(int, grid.split("x"))
        outs = _run_ranks(exe, [grid, "384", "32", warm], p * q, timeout=120)
        first = [l for l in outs[0][1].splitlines() if l.startswith("rep 0")]
        print(f"iter {it} {grid} warm={warm} {v} rc={[o[0] for o in outs]} {first}", flush=True)
