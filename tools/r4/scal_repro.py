import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from tests.test_native_gpu import _run_ranks, ROOT
exe = os.path.join(ROOT, "slate_amd", "scal_probe")
variants = [{}, {"SLATE_AMD_NATIVE_SERIAL": "1"}, {"SLATE_AMD_POTRF_CHUNK": "100"}]
for it in range(int(sys.argv[1])):
    for v in variants:
        for k in ("SLATE_AMD_NATIVE_SERIAL", "SLATE_AMD_POTRF_CHUNK"):
            os.environ.pop(k, None)
        os.environ.update(v)
        outs = _run_ranks(exe, ["2x2", "384", "32"], 4, timeout=120)
        first = [l for l in outs[0][1].splitlines() if l.startswith("rep 0")]
        print(f"iter {it} {v} rc={[o[0] for o in outs]} {first}", flush=True)
