"""Project the 8-GPU (p x q) critical path of dpotrf / dgemm from ONE GPU.

One process plays world rank r of the p x q job through the loopback
transport (slate_amd/parallel/comm.py LoopbackComm): the rank's own kernel
DAG runs at its true local shapes and stream order, and every collective is
a same-size local device copy on its issuing stream.  The communication is
then priced from the logged (op, communicator size, bytes, stream) records
under stated xGMI / RCCL assumptions:

  T_rank = T_loopback + sum over collectives issued from the panel / diag
           streams (the factorization's chain) of alpha + bytes / beta
           (+ the update-stream collectives too in the pessimistic column,
           i.e. none of them hidden behind the trailing GEMMs)

The job time is the max over the simulated ranks.  Data received through
the loopback is the rank's own bytes, not its peers' (kernel timings here
are data-independent: no early exits in the tile kernels).

    python tools/r5/loopback_critpath.py [--routine potrf] [--n 32768] [--nb 512]
        [--grid 2x4] [--ranks 0,1,5] [--lookahead 1] [--out profiles/r5/critpath_2x4.md]
"""
import argparse
import collections
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

# (alpha seconds per collective, beta bytes / second effective per collective)
SCENARIOS = {
    "optimistic": (10e-6, 150e9),     # one xGMI link's rate, RCCL small-message latency
    "pessimistic": (25e-6, 50e9),     # ring bcast over 4 GPUs, one third of a link each hop
}
PEAK = 78.6e12                         # fp64 matrix peak per MI355X


def run_rank(args, r, p, q):
    import slate_amd as sl
    from slate_amd.parallel import comm as C
    from slate_amd.parallel.streams import _SHARED
    C.loopback(p * q, r)
    gpu = torch.cuda.is_available()
    dev = torch.device("cuda", 0) if gpu else torch.device("cpu")
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    n, nb = args.n, args.nb
    opts = {sl.Option.Lookahead: args.lookahead, sl.Option.Target: sl.Target.Devices if gpu else sl.Target.HostTask}
    if args.routine == "potrf":
        A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, p=p, q=q, device=dev)
        A.insertLocalTiles(device=dev)
        sl.generate_matrix(A, "poev", seed=7)
        run = lambda: sl.potrf(A, opts)          # noqa: E731
        flops = n ** 3 / 3
    elif args.routine == "getrf":
        A = sl.Matrix(n, n, nb=nb, p=p, q=q, device=dev)
        A.insertLocalTiles(device=dev)
        sl.generate_matrix(A, "rands", seed=7)
        run = lambda: sl.getrf(A, sl.Pivots(), opts)     # noqa: E731
        flops = 2 * n ** 3 / 3
    else:
        A = sl.Matrix(n, n, nb=nb, p=p, q=q, device=dev)
        A.insertLocalTiles(device=dev)
        sl.generate_matrix(A, "rands", seed=7)
        B = sl.Matrix(n, n, nb=nb, p=p, q=q, device=dev)
        B.insertLocalTiles(device=dev)
        sl.generate_matrix(B, "rands", seed=8)
        Cm = sl.Matrix(n, n, nb=nb, p=p, q=q, device=dev)
        Cm.insertLocalTiles(device=dev)
        run = lambda: sl.gemm(1.0, A, B, 0.0, Cm, opts)   # noqa: E731
        flops = 2.0 * n ** 3
    local = A.storage.local[A.storage.origin_slot]
    backup = local.clone()

    def step():
        local.copy_(backup)
        A.storage.mark_local_modified(A.storage.origin_slot)
        return run()

    step()
    sync()
    times, logs = [], []
    for _ in range(args.steps):
        C.LoopbackComm.LOG.clear()
        sync()
        t0 = time.perf_counter()
        step()
        sync()
        times.append(time.perf_counter() - t0)
        logs.append(list(C.LoopbackComm.LOG))
    sh = _SHARED.get(str(dev), {})
    names = {}
    for key, label in (("panel", "panel"), ("diag", "diag")):
        st = sh.get(key)
        if st is not None:
            names[st.cuda_stream] = label
    if "upd" in sh:
        names[sh["upd"][1].cuda_stream] = "update"
    best = min(range(len(times)), key=lambda i: times[i])
    log = logs[best]
    agg = collections.defaultdict(lambda: [0, 0])
    for op, size, nbytes, st in log:
        k = (names.get(st, "other"), op, size)
        agg[k][0] += 1
        agg[k][1] += nbytes
    pr, pc = r % p, r // p
    return dict(rank=r, pr=pr, pc=pc, t=times[best], flops=flops, agg=dict(agg),
                mloc=local.shape[0], nloc=local.shape[1])


def model(res, scen):
    alpha, beta = SCENARIOS[scen]
    chain = sum(c * alpha + b / beta for (st, op, size), (c, b) in res["agg"].items() if st != "update")
    upd = sum(c * alpha + b / beta for (st, op, size), (c, b) in res["agg"].items() if st == "update")
    return chain, upd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--routine", default="potrf", choices=["potrf", "getrf", "gemm"])
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--nb", type=int, default=512)
    ap.add_argument("--grid", default="2x4")
    ap.add_argument("--ranks", default="0,1,5")
    ap.add_argument("--lookahead", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--out", default=None)
    ap.add_argument("--link", default=None,
                    help="alpha_us,beta_GBps: model every collective IN the DAG (a spin kernel of its "
                         "duration on its issuing stream, parallel/comm.py LoopbackComm) and report the "
                         "measured time as the projection")
    args = ap.parse_args()
    p, q = map(int, args.grid.lower().split("x"))
    if args.link:
        from slate_amd.parallel.comm import LoopbackComm
        os.environ["SLATE_AMD_LOOPBACK_LINK"] = args.link
        LoopbackComm._link = None
    res = [run_rank(args, int(r), p, q) for r in args.ranks.split(",")]
    if args.link:
        a_us, b_gb = args.link.split(",")[:2]
        lines = [f"## {args.routine} n={args.n} nb={args.nb} grid {p}x{q} lookahead {args.lookahead}: in-DAG link "
                 f"model alpha {a_us} us, beta {b_gb} GB/s (loopback, 1 MI355X)", ""]
        worst = max(x["t"] for x in res)
        for x in res:
            lines.append(f"- rank {x['rank']} ({x['pr']},{x['pc']}): {x['t'] * 1e3:.1f} ms")
        fl = res[0]["flops"]
        lines.append(f"- job (max over simulated ranks): {worst * 1e3:.1f} ms = {fl / worst / 1e12:.1f} TF/s "
                     f"({100 * fl / worst / (p * q * PEAK):.1f} % of {p * q} x 78.6)")
        # per-link accounting: the bytes each collective puts on its BUSIEST
        # link (ring / pipelined bcast, reduce: the message; allreduce: 2x;
        # all-gather: (size - 1)x; the direct bcast_sa: 2 / size of it)
        from slate_amd.parallel.comm import LoopbackComm
        for x in res:
            for (st, op, size), (c, b) in sorted(x["agg"].items()):
                f = (2.0 / size) if op == "bcast_sa" else LoopbackComm._LINK_FACTOR.get(op, float(size - 1))
                lines.append(f"  - rank {x['rank']}: {st} {op} over {size}: {c} calls, {b / 2 ** 20:.1f} MiB, "
                             f"busiest link {f * b / 2 ** 20:.1f} MiB")
        text = "\n".join(lines)
        print(text, flush=True)
        if args.out:
            with open(args.out, "a") as f:
                f.write(text + "\n\n")
        return
    lines = [f"## {args.routine} n={args.n} nb={args.nb} grid {p}x{q} lookahead {args.lookahead} (loopback, 1 MI355X)", ""]
    lines.append("| rank (pr,pc) | local block | loopback ms | chain comm ms (opt / pess) | update comm ms (opt / pess) |"
                 " projected ms (opt / pess) | projected TF/s job (opt / pess) | % of 8-GPU peak (opt / pess) |")
    lines.append("|---|---|---|---|---|---|---|---|")
    worst = {"optimistic": 0.0, "pessimistic": 0.0}
    for x in res:
        co, uo = model(x, "optimistic")
        cp, up = model(x, "pessimistic")
        to = x["t"] + co
        tp = x["t"] + cp + up
        worst["optimistic"] = max(worst["optimistic"], to)
        worst["pessimistic"] = max(worst["pessimistic"], tp)
        lines.append(f"| {x['rank']} ({x['pr']},{x['pc']}) | {x['mloc']}x{x['nloc']} | {x['t'] * 1e3:.1f} | "
                     f"{co * 1e3:.1f} / {cp * 1e3:.1f} | {uo * 1e3:.1f} / {up * 1e3:.1f} | {to * 1e3:.1f} / {tp * 1e3:.1f} | "
                     f"{x['flops'] / to / 1e12:.1f} / {x['flops'] / tp / 1e12:.1f} | "
                     f"{100 * x['flops'] / to / (p * q * PEAK):.1f} / {100 * x['flops'] / tp / (p * q * PEAK):.1f} |")
    fl = res[0]["flops"]
    lines.append("")
    lines.append(f"Job projection (max over the simulated ranks): optimistic {worst['optimistic'] * 1e3:.1f} ms = "
                 f"{fl / worst['optimistic'] / 1e12:.1f} TF/s ({100 * fl / worst['optimistic'] / (p * q * PEAK):.1f} % of "
                 f"{p * q} x 78.6); pessimistic {worst['pessimistic'] * 1e3:.1f} ms = {fl / worst['pessimistic'] / 1e12:.1f} TF/s "
                 f"({100 * fl / worst['pessimistic'] / (p * q * PEAK):.1f} %).")
    lines.append("")
    lines.append("Collectives per factorization (rank, stream, op, communicator size: count, MiB):")
    lines.append("")
    for x in res:
        for (st, op, size), (c, b) in sorted(x["agg"].items()):
            lines.append(f"- rank {x['rank']}: {st} {op} over {size}: {c} calls, {b / 2 ** 20:.1f} MiB")
    text = "\n".join(lines)
    print(text, flush=True)
    if args.out:
        with open(args.out, "a") as f:
            f.write(text + "\n\n")


if __name__ == "__main__":
    main()
