"""Accuracy sweep of the native grid heev (bench_native heev check) over n
and grid shapes, host transport on one GPU."""
import sys
sys.path.insert(0, __import__("os").path.dirname(__file__))
from heev_grid_bench import run  # noqa: E402

for (p, q) in ((2, 1), (1, 2), (2, 2), (1, 4)):
    for n in (512, 1024, 2048):
        for mode in ("grid",):
            rc, out = run(["heev", str(n), "256", str(p), str(q), "1", "0", "1", "1"], p * q,
                          {"SLATE_AMD_NATIVE_HEEV": mode})
            res = [l for l in out.splitlines() if "RESULT" in l or "rror" in l]
            print(f"{p}x{q} n={n} {mode}: rc={rc}", *res, flush=True)
