"""Run every tester routine once in ONE process (GPU box friendly):
python tools/tester_all.py [--dim 300] [--nb 64] [--type d,z] [--target d]"""
import argparse
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from slate_amd import tester  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", default="300")
    ap.add_argument("--nb", default="64")
    ap.add_argument("--type", default="d,z")
    ap.add_argument("--target", default="d")
    a = ap.parse_args()
    bad = []
    for r in sorted(tester.ROUTINES):
        t0 = time.time()
        rc = tester.main([r, "--type", a.type, "--dim", a.dim, "--nb", a.nb, "--target", a.target])
        print(f"== {r}: {'ok' if rc == 0 else 'FAILED'} ({time.time() - t0:.1f} s)", flush=True)
        if rc:
            bad.append(r)
    print("FAILED:", bad if bad else "none", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
