import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from tests.test_native_gpu import _run_ranks, ROOT
exe = os.path.join(ROOT, "slate_amd", "scal_probe")
os.environ["SLATE_AMD_NATIVE_TRACE"] = "1"
outs = _run_ranks(exe, ["2x1", "128", "32", "0"], 2, timeout=120)
for r, (rc, o) in enumerate(outs):
    print(f"=== rank {r} rc={rc}")
    print(o)
