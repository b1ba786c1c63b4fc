"""Trailing-update GEMM efficiency of the distributed dpotrf on a 1 x q / p x q
grid vs the one-rank path, step by step: the exact masked GEMM rank (pr, pc)
runs at step t (C = local rows >= tile t+1, local columns past the lookahead),
timed alone, priced at its kept (lower-triangle) flops.

    python tools/r5/stair_probe.py [--grid 1x2] [--n 32768] [--nb 512] [--steps 0,8,16,32,48]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from slate_amd import ops


def tlb(g, p, r):
    return (g - r + p - 1) // p if g > r else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", default="1x2")
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--nb", type=int, default=512)
    ap.add_argument("--K", type=int, default=0)
    ap.add_argument("--steps", default="0,8,16,32,48")
    ap.add_argument("--la", type=int, default=1)
    a = ap.parse_args()
    p, q = map(int, a.grid.split("x"))
    n, nb, la = a.n, a.nb, a.la
    K = a.K or nb
    nt = n // nb
    dev = torch.device("cuda", 0)
    cm = lambda m, k: torch.randn(k, m, dtype=torch.float64, device=dev).t()   # noqa: E731
    pr, pc = 0, 0
    mloc, nloc = tlb(nt, p, pr) * nb, tlb(nt, q, pc) * nb
    buf = cm(mloc, nloc)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    print(f"grid {p}x{q} rank (0,0) local {mloc}x{nloc} K={K}")
    for t in map(int, a.steps.split(",")):
        g = t
        lr1 = tlb(g + 1, p, pr) * nb
        lc_la = tlb(g + 1 + la, q, pc) * nb
        nrow = mloc - lr1
        ncol = nloc - lc_la
        if nrow <= 0 or ncol <= 0:
            continue
        P = cm(nrow, K)
        L = cm(ncol, K)
        C = buf[lr1:, lc_la:]
        mask = (1, nb, p, pr, q, pc, lr1, lc_la, 0)
        kept = 0
        for jl in range(lc_la // nb, nloc // nb):
            jg = jl * q + pc
            for il in range(lr1 // nb, mloc // nb):
                ig = il * p + pr
                if ig >= jg:
                    kept += 1
        fl = 2.0 * kept * nb * nb * K
        fn = lambda: ops.gemm(-1.0, P, L, 1.0, C, 'N', 'T', mask)   # noqa: E731
        fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        # the one-rank equivalent: a dense lower-staircase with the same kept tiles
        print(f"step {t:3d}: C {nrow}x{ncol} kept {kept} tiles ({100 * kept * nb * nb / (nrow * ncol):.0f}%) "
              f"{ms:.3f} ms {fl / ms / 1e9:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
