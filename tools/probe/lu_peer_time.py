"""Host issue time of the distributed LU panel, peer-mailbox form against the
host-issued record all-gather form (<= 0.3 ms of host
time per 512-column panel at 2 x 1).  Two ranks share cuda:0 over gloo, so
the device times are a rehearsal only; the host issue time per panel is what
one rank's driver thread spends inside `_panel_pp_dist`.

    python tools/probe/lu_peer_time.py [n] [nb]
"""
import os
import sys
import time

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _rank(rank, size, port, n, nb, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(size),
                      LOCAL_RANK=str(rank), SLATE_AMD_LU_PANEL_GATHER="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=size)
    import slate_amd as sl
    from slate_amd.models import lu as lu_mod
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    orig = lu_mod._panel_pp_dist
    acc = {"t": 0.0, "n": 0}

    def timed(*a, **k):
        t0 = time.perf_counter()
        r = orig(*a, **k)
        acc["t"] += time.perf_counter() - t0
        acc["n"] += 1
        return r
    lu_mod._panel_pp_dist = timed
    res = {}
    for mode in ("0", "1", "0", "1"):
        os.environ["SLATE_AMD_LU_PEER"] = mode
        A = sl.Matrix(n, n, nb=nb, p=size, q=1, device=dev)
        A.insertLocalTiles(device=0)
        sl.generate_matrix(A, "rands", 3)
        piv = sl.Pivots()
        acc["t"], acc["n"] = 0.0, 0
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        info = sl.getrf(A, piv, {sl.Option.Lookahead: 1})
        torch.cuda.synchronize()
        dist.barrier()
        wall = time.perf_counter() - t0
        res[mode] = (wall, acc["t"] / max(acc["n"], 1), acc["n"], info)
    if rank == 0:
        for mode, (wall, per, cnt, info) in res.items():
            form = "peer mailbox" if mode == "1" else "record all-gather"
            print(f"n={n} nb={nb} 2x1 on one GPU, {form:18s}: getrf {wall * 1e3:8.1f} ms, "
                  f"host time in the panel {per * 1e3:7.3f} ms per panel ({cnt} panels), info {info}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_rank, args=(2, port, n, nb, 1), nprocs=2, join=True)
