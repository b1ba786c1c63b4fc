"""Direct two-phase broadcast (Comm.bcast_sa: scatter + all-gather over
grouped point-to-point) on gloo ranks, and the 1 x q / 2 x q Cholesky with
its row broadcasts switched to it (SLATE_AMD_BCAST_SA=1)."""
import os

import pytest
import torch

from dist_util import run_dist


def _bsa(rank, size):
    from slate_amd.parallel.comm import world
    w = world()
    for n, m, root in ((37, 5, 0), (1, 1, 2), (64, 3, size - 1), (7, 2, 1)):
        ref = torch.arange(n * m, dtype=torch.float64).reshape(m, n).t() * 0.5 + 3 * root
        t = torch.empty(m, n, dtype=torch.float64).t()        # column-major n x m
        if w.rank == root:
            t.copy_(ref)
        else:
            t.fill_(-1)
        w.bcast_sa(t, root)
        assert torch.equal(t, ref), (rank, n, m, root)
    # a strided (non-contiguous) view falls back to a contiguous copy
    big = torch.zeros(10, 6, dtype=torch.float64)
    v = big[1:9, 2:5]
    if w.rank == 0:
        v.copy_(torch.arange(24, dtype=torch.float64).reshape(8, 3))
    w.bcast_sa(v, 0)
    assert torch.equal(v, torch.arange(24, dtype=torch.float64).reshape(8, 3))


def test_bcast_sa_gloo():
    run_dist(_bsa, 4)


def _potrf(rank, size, p, q):
    os.environ["SLATE_AMD_BCAST_SA"] = "1"
    import slate_amd as sl
    from slate_amd.models import chol
    chol._BCAST_SA = True
    n, nb = 200, 16
    A = sl.HermitianMatrix(sl.Uplo.Lower, n, nb=nb, p=p, q=q)
    A.insertLocalTiles()
    sl.generate_matrix(A, "poev", seed=3)
    from slate_amd.models.aux import allgather_dense
    F = allgather_dense(A).clone()
    F = torch.tril(F) + torch.tril(F, -1).mT
    info = sl.potrf(A)
    L = torch.tril(allgather_dense(A))
    assert info == 0
    err = (L @ L.mT - F).norm() / F.norm()
    assert err < 1e-13, err


@pytest.mark.parametrize("grid", [(1, 4), (1, 3)])
def test_potrf_rows_bcast_sa(grid):
    run_dist(_potrf, grid[0] * grid[1], *grid)
