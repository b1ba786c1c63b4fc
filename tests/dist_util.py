"""Multi-process (gloo, 127.0.0.1) harness for the distributed drivers.

``run_dist(fn, nprocs)`` spawns nprocs ranks that initialise
torch.distributed with the gloo backend and call ``fn(rank, size)``; an
exception on any rank fails the test with that rank's traceback.  ``fn``
must be a module-level function (spawn pickles it by reference).
"""
import os
import socket
import traceback

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, size, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(size), LOCAL_RANK=str(rank))
    try:
        import torch
        import torch.distributed as dist
        torch.set_num_threads(2)
        dist.init_process_group("gloo", rank=rank, world_size=size)
        try:
            fn(rank, size, *args)
        finally:
            from slate_amd.parallel import comm as _c
            _c.ProcessGrid._cache.clear()
            dist.destroy_process_group()
        q.put((rank, None))
    except BaseException:  # noqa: BLE001
        q.put((rank, traceback.format_exc()))


def run_dist(fn, nprocs=2, *args, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, nprocs, port, fn, args, q)) for r in range(nprocs)]
    for p in procs:
        p.start()
    errs = {}
    try:
        for _ in range(nprocs):
            rank, err = q.get(timeout=timeout)
            if err:
                errs[rank] = err
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    if errs:
        msg = "\n".join(f"rank {r} failed:\n{errs[r]}" for r in sorted(errs))
        raise AssertionError(msg)
