"""Cross-communicator issue order of the pipelined drivers (VERDICT r5 next
#1: "give every RCCL communicator a fixed issue order across ranks").

Each rank logs, in issue order, the (communicator, sequence number) of every
collective and matched point-to-point pair it takes part in
(``parallel.comm.ORDER_LOG``).  The union of the per-rank chains must be
acyclic: then one global order of all collectives exists of which every
rank's issue order is a restriction, and no sharing of hardware queues
between the streams that carry different communicators can deadlock
(argument in the parallel/comm.py docstring).  Also checked: every member of
a communicator issued the same number of operations on it, of the same kinds.
The host issue order of a driver does not depend on the device (the CPU
runs use gloo, the GPU runs RCCL, through the same driver code).
"""
import json
import os
import tempfile
from collections import defaultdict

import pytest
import torch

import slate_amd as sl
from slate_amd.core.enums import Option

from dist_util import run_dist


def _drive(routine, p, q, n, nb):
    opts = {Option.Lookahead: 1}
    if routine == "potrf":
        A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, p=p, q=q)
        A.insertLocalTiles()
        sl.generate_matrix(A, "poev", seed=3)
        assert sl.potrf(A, opts) == 0
    elif routine == "getrf":
        A = sl.Matrix(n, n, nb=nb, p=p, q=q)
        A.insertLocalTiles()
        sl.generate_matrix(A, "rands", seed=3)
        opts[Option.Lookahead] = 2
        assert sl.getrf(A, sl.Pivots(), opts) == 0
    elif routine == "geqrf":
        A = sl.Matrix(n + n // 2, n, nb=nb, p=p, q=q)
        A.insertLocalTiles()
        sl.generate_matrix(A, "rands", seed=3)
        sl.geqrf(A, sl.TriangularFactors(), opts)
    elif routine == "gemm":
        mk = []
        for s in range(3):
            X = sl.Matrix(n, n, nb=nb, p=p, q=q)
            X.insertLocalTiles()
            sl.generate_matrix(X, "rands", seed=s)
            mk.append(X)
        sl.gemm(1.0, mk[0], mk[1], 0.0, mk[2], opts)
    elif routine == "heev":
        A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, p=p, q=q)
        A.insertLocalTiles()
        sl.generate_matrix(A, "rands", seed=3)
        Z = sl.Matrix(n, n, nb=nb, p=p, q=q)
        Z.insertLocalTiles()
        sl.heev(A, None, Z, opts)


def _worker(rank, size, routine, p, q, n, nb, outdir):
    from slate_amd.parallel import comm as C
    C.ORDER_LOG.update(on=True, ops=[], seq={})
    try:
        _drive(routine, p, q, n, nb)
    finally:
        C.ORDER_LOG["on"] = False
    ops = [[list(map(list, [k[0]])) + list(k[1:]), kind, s] for k, kind, s in C.ORDER_LOG["ops"]]
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump(ops, f)


def _check(logs):
    """logs: rank -> [(key, kind, seq)].  Returns the number of nodes."""
    kinds = {}
    count = defaultdict(dict)
    succ = defaultdict(set)
    indeg = defaultdict(int)
    nodes = set()
    for r, ops in logs.items():
        prev = None
        for key, kind, s in ops:
            key = json.dumps(key)
            node = (key, s)
            if node in kinds:
                assert kinds[node] == kind, f"rank {r}: {node} is {kind} here, {kinds[node]} elsewhere"
            kinds[node] = kind
            count[key][r] = count[key].get(r, 0) + 1
            nodes.add(node)
            if prev is not None and node not in succ[prev]:
                succ[prev].add(node)
                indeg[node] += 1
            prev = node
    for key, per in count.items():
        assert len(set(per.values())) == 1, f"members of {key} issued different counts: {per}"
    # Kahn: every node must be removable
    ready = [x for x in nodes if indeg[x] == 0]
    seen = 0
    while ready:
        x = ready.pop()
        seen += 1
        for y in succ[x]:
            indeg[y] -= 1
            if indeg[y] == 0:
                ready.append(y)
    assert seen == len(nodes), f"issue orders form a cycle ({len(nodes) - seen} collectives on it)"
    return len(nodes)


@pytest.mark.parametrize("routine,p,q", [
    ("potrf", 2, 2), ("potrf", 2, 4), ("getrf", 2, 2), ("getrf", 2, 4), ("geqrf", 2, 2),
    ("gemm", 2, 2), ("heev", 2, 2)])
def test_issue_order_acyclic(routine, p, q):
    n, nb = (192, 16) if routine != "heev" else (96, 16)
    with tempfile.TemporaryDirectory() as d:
        run_dist(_worker, p * q, routine, p, q, n, nb, d, timeout=600)
        logs = {}
        for r in range(p * q):
            with open(os.path.join(d, f"r{r}.json")) as f:
                logs[r] = [(k, kind, s) for k, kind, s in json.load(f)]
    assert sum(len(v) for v in logs.values()) > 0
    _check(logs)


def test_checker_finds_a_crossed_order():
    """Two ranks issuing two communicators' collectives in opposite orders
    are reported as a cycle."""
    a, b = [[0, 1], ""], [[0, 1], "update"]
    logs = {0: [(a, "bcast", 0), (b, "bcast", 0)], 1: [(b, "bcast", 0), (a, "bcast", 0)]}
    with pytest.raises(AssertionError, match="cycle"):
        _check(logs)
    logs = {0: [(a, "bcast", 0), (b, "bcast", 0)], 1: [(a, "bcast", 0), (b, "bcast", 0)]}
    assert _check(logs) == 2
