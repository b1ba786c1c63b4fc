"""Native heev timings: 1 GPU (n = 16384) and 2x2 over the host transport
on one GPU (grid vs gather path, peak device memory per rank).  Prints one
line per run; used by tools/r6/gpu_u.sh."""
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
EXE = os.path.join(ROOT, "slate_amd", "bench_native")


def env(rank=None, size=None, port=None, extra=None):
    e = {k: v for k, v in os.environ.items() if not k.startswith("PYTHON")}
    e["LD_LIBRARY_PATH"] = "/opt/rocm/lib"
    if rank is not None:
        e.update(RANK=str(rank), WORLD_SIZE=str(size), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                 MASTER_PORT=str(port), SLATE_AMD_NATIVE_TRANSPORT="host")
    e.update(extra or {})
    return e


def run(args, nranks=1, extra=None, timeout=600):
    if nranks == 1:
        r = subprocess.run([EXE] + args, capture_output=True, text=True, env=env(extra=extra), timeout=timeout)
        return r.returncode, r.stdout + r.stderr
    port = random.randint(20000, 50000)
    ps = [subprocess.Popen([EXE] + args, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           env=env(r, nranks, port, extra)) for r in range(nranks)]
    outs = [p.communicate(timeout=timeout)[0] for p in ps]
    return max(p.returncode for p in ps), "".join(outs)


def main():
    which = sys.argv[1:] or ["1gpu", "grid"]
    if "1gpu" in which:
        for n in (8192, 16384):
            rc, out = run(["heev", str(n), "256", "1", "1", "1", "1", "2", "1"])
            print(f"1x1 n={n}:", rc, [l for l in out.splitlines() if "RESULT" in l or "error" in l.lower()], flush=True)
    if "grid" in which:
        for mode in ("grid", "gather"):
            extra = {"SLATE_AMD_NATIVE_MEMREPORT": "1"}
            if mode == "gather":
                extra["SLATE_AMD_NATIVE_HEEV"] = "gather"
            rc, out = run(["heev", "4096", "256", "2", "2", "1", "1", "1", "1"], 4, extra)
            keep = [l for l in out.splitlines() if "RESULT" in l or "peak" in l or "rror" in l]
            print(f"2x2 n=4096 {mode}:", rc, *keep, sep="\n  ", flush=True)


if __name__ == "__main__":
    main()
