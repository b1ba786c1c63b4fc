"""Distributed parallel BLAS-3 and redistribution without dense gathers.

Reference strategy: test/test_gemm.cc, test_herk.cc, test_hemm.cc,
test_trmm.cc, test_trsm.cc (randomised residual checks on every grid) and
unit_test/test_Matrix.cc (redistribute / views).  The oracle here is PyTorch
fp64 on the gathered matrices (test-side only); the library paths under test
never gather (parallel/redist.py, models/blas3.py).

Grids: 1x1 in-process, and gloo ranks on 2x1, 1x2, 2x2, 2x4 (8 ranks).
"""
import pytest
import torch

import slate_amd as sl
from slate_amd.core.enums import Diag, MethodGemm, MethodHemm, MethodTrsm, Op, Option, Side, Uplo
from slate_amd.models.aux import allgather_dense as D

from dist_util import run_dist


def mat(m, n, nb, seed, p, q, dt=torch.float64):
    A = sl.Matrix(m, n, nb=nb, p=p, q=q, dtype=dt)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rands", seed)
    return A


def herm(n, nb, seed, p, q, dt=torch.float64, uplo=Uplo.Lower, cls=sl.HermitianMatrix):
    A = cls(uplo, n, nb=nb, p=p, q=q, dtype=dt)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rands", seed)
    return A


def close(a, b, tol=1e-11):
    s = max(1.0, b.abs().max().item())
    err = (a - b).abs().max().item() / s
    assert err <= tol, err


def tri(X, uplo):
    return torch.tril(X) if uplo == Uplo.Lower else torch.triu(X)


def full(Hd, uplo, herm_=True):
    L = tri(Hd, uplo)
    M = L.mH if herm_ else L.T
    F = L + M - torch.diag(torch.diagonal(L))
    if herm_ and F.is_complex():
        F.diagonal().imag.zero_()
    return F


def opx(X, op):
    return X if op == Op.NoTrans else (X.T if op == Op.Trans else X.mH)


def view(X, op):
    return X if op == Op.NoTrans else (X.transpose() if op == Op.Trans else X.conj_transpose())


# -------------------------------------------------------------------- checks
def check_redistribute(p, q, dt=torch.float64):
    A = mat(70, 45, 16, 1, p, q, dt)
    Ad = D(A)
    # different tile size, transposed grid, transposed / conj-transposed source
    for op in (Op.NoTrans, Op.Trans, Op.ConjTrans):
        src = view(A, op)
        B = sl.Matrix(src.m(), src.n(), nb=12, p=q, q=p, dtype=dt)
        B.insertLocalTiles()
        sl.redistribute(src, B)
        close(D(B), opx(Ad, op), 0)
    # sub-view to sub-view with offsets that are not tile aligned
    B = mat(70, 45, 8, 2, q, p, dt)
    Bd = D(B)
    sl.redistribute(A.slice(5, 40, 3, 30), B.slice(10, 45, 7, 34))
    Bd[10:46, 7:35] = Ad[5:41, 3:31]
    close(D(B), Bd, 0)


def check_conj_transpose_keeps_other_triangle(p, q, dt=torch.float64):
    H = herm(50, 16, 3, p, q, dt, Uplo.Upper)
    Hd = D(H)
    L = sl.HermitianMatrix(Uplo.Lower, 50, nb=16, p=p, q=q, dtype=dt)
    L.insertLocalTiles()
    sl.set(77.0, 77.0, sl.Matrix(_storage=L.storage))
    sl.copy_conj_transpose(H, L)
    Ld = D(L)
    close(torch.tril(Ld), torch.tril(torch.triu(Hd).mH), 0)
    # strictly upper part of L untouched
    assert bool((torch.triu(Ld, 1) == torch.triu(torch.full_like(Ld, 77.0), 1)).all())


def check_potrf_upper_keeps_lower(p, q, dt=torch.float64):
    n, nb = 64, 16
    A = sl.HermitianMatrix(Uplo.Upper, n, nb=nb, p=p, q=q, dtype=dt)
    A.insertLocalTiles()
    sl.generate_matrix(A, "poev", 5)
    G = sl.Matrix(_storage=A.storage)
    Gd = D(G)
    # poison the unreferenced (strictly lower) triangle
    Pd = torch.triu(Gd) + torch.tril(torch.full_like(Gd, 77.0), -1)
    sl.from_dense(G, Pd)
    Af = full(torch.triu(Gd), Uplo.Upper)
    assert sl.potrf(A) == 0
    F = D(G)
    U = torch.triu(F)
    close(U.mH @ U, Af, 1e-12)
    assert bool((torch.tril(F, -1) == torch.tril(torch.full_like(F, 77.0), -1)).all())


def check_gemm_all(p, q, dt=torch.float64):
    for ta in (Op.NoTrans, Op.Trans, Op.ConjTrans):
        for tb in (Op.NoTrans, Op.ConjTrans):
            A = mat(50, 37, 16, 4, p, q, dt) if ta == Op.NoTrans else mat(37, 50, 16, 4, p, q, dt)
            B = mat(37, 41, 16, 5, p, q, dt) if tb == Op.NoTrans else mat(41, 37, 16, 5, p, q, dt)
            C = mat(50, 41, 16, 6, p, q, dt)
            Ad, Bd, Cd = D(A), D(B), D(C)
            sl.gemm(1.25, view(A, ta), view(B, tb), -0.5, C)
            close(D(C), 1.25 * opx(Ad, ta) @ opx(Bd, tb) - 0.5 * Cd)
    # different tile sizes / grids for the operands, C is a sub-view
    A = sl.Matrix(40, 33, nb=10, p=q, q=p, dtype=dt)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rands", 7)
    B = mat(33, 29, 16, 8, p, q, dt)
    C = mat(60, 50, 16, 9, p, q, dt)
    Ad, Bd, Cd = D(A), D(B), D(C)
    sl.gemm(2.0, A, B, 1.0, C.slice(3, 42, 5, 33))
    Cd[3:43, 5:34] += 2.0 * Ad @ Bd
    close(D(C), Cd)


def check_gemmA(p, q, dt=torch.float64):
    # skinny B / C: stationary A with reduce (auto for one block column) and forced
    for method, nrhs in ((MethodGemm.Auto, 7), (MethodGemm.A, 40)):
        A = mat(70, 66, 16, 10, p, q, dt)
        B = mat(66, nrhs, 16, 11, p, q, dt)
        C = mat(70, nrhs, 16, 12, p, q, dt)
        Ad, Bd, Cd = D(A), D(B), D(C)
        sl.gemm(1.5, A, B, 0.25, C, {Option.MethodGemm: method})
        close(D(C), 1.5 * Ad @ Bd + 0.25 * Cd)


def check_rank_k(p, q, dt=torch.float64):
    for uplo in (Uplo.Lower, Uplo.Upper):
        for trans in (Op.NoTrans, Op.ConjTrans):
            for sym in (False, True):
                if sym and trans == Op.ConjTrans and dt.is_complex:
                    continue
                cls = sl.SymmetricMatrix if sym else sl.HermitianMatrix
                A = mat(45, 21, 16, 13, p, q, dt) if trans == Op.NoTrans else mat(21, 45, 16, 13, p, q, dt)
                B = mat(45, 21, 16, 14, p, q, dt) if trans == Op.NoTrans else mat(21, 45, 16, 14, p, q, dt)
                C = herm(45, 16, 15, p, q, dt, uplo, cls)
                G = sl.Matrix(_storage=C.storage)
                Cd = D(G)
                Ao = view(A, trans if not sym else (Op.Trans if trans != Op.NoTrans else Op.NoTrans))
                Bo = view(B, trans if not sym else (Op.Trans if trans != Op.NoTrans else Op.NoTrans))
                a, b = opx(D(A), Ao.op()), opx(D(B), Bo.op())
                H = (lambda X: X.T) if sym else (lambda X: X.mH)
                if sym:
                    sl.syrk(0.5, Ao, 2.0, C)
                    ref = 0.5 * a @ H(a) + 2.0 * full(Cd, uplo, False)
                else:
                    sl.herk(0.5, Ao, 2.0, C)
                    ref = 0.5 * a @ H(a) + 2.0 * full(Cd, uplo)
                out = D(G)
                close(tri(out, uplo), tri(ref, uplo))
                # the other triangle is never written
                other = Uplo.Upper if uplo == Uplo.Lower else Uplo.Lower
                strict = (lambda X: torch.triu(X, 1)) if other == Uplo.Upper else (lambda X: torch.tril(X, -1))
                assert bool((strict(out) == strict(Cd)).all())
                C2 = herm(45, 16, 16, p, q, dt, uplo, cls)
                G2 = sl.Matrix(_storage=C2.storage)
                C2d = D(G2)
                if sym:
                    sl.syr2k(0.75, Ao, Bo, -1.0, C2)
                    ref = 0.75 * (a @ H(b) + b @ H(a)) - full(C2d, uplo, False)
                else:
                    sl.her2k(0.75, Ao, Bo, -1.0, C2)
                    ref = 0.75 * a @ H(b) + 0.75 * b @ H(a) - full(C2d, uplo)
                close(tri(D(G2), uplo), tri(ref, uplo))


def check_hemm(p, q, dt=torch.float64):
    for side in (Side.Left, Side.Right):
        for uplo in (Uplo.Lower, Uplo.Upper):
            for sym in (False, True):
                cls = sl.SymmetricMatrix if sym else sl.HermitianMatrix
                A = herm(36, 16, 17, p, q, dt, uplo, cls)
                Afull = full(D(sl.Matrix(_storage=A.storage)), uplo, not sym)
                B = mat(36, 22, 16, 18, p, q, dt) if side == Side.Left else mat(22, 36, 16, 18, p, q, dt)
                C = mat(B.m(), B.n(), 16, 19, p, q, dt)
                Bd, Cd = D(B), D(C)
                (sl.symm if sym else sl.hemm)(side, 1.5, A, B, 0.5, C)
                ref = 1.5 * (Afull @ Bd if side == Side.Left else Bd @ Afull) + 0.5 * Cd
                close(D(C), ref)


def check_trmm_trsm(p, q, dt=torch.float64):
    n = 40
    T = mat(n, n, 16, 20, p, q, dt)
    Td = D(T) + 4.0 * torch.eye(n, dtype=dt)
    sl.from_dense(T, Td)
    for side in (Side.Left, Side.Right):
        for uplo in (Uplo.Lower, Uplo.Upper):
            for op in (Op.NoTrans, Op.Trans, Op.ConjTrans):
                for diag in (Diag.NonUnit, Diag.Unit):
                    Tv = view(sl.TriangularMatrix(uplo, T, diag=diag), op)
                    Tl = tri(Td, uplo)
                    if diag == Diag.Unit:
                        Tl = Tl - torch.diag(torch.diagonal(Tl)) + torch.eye(n, dtype=dt)
                    Tl = opx(Tl, op)
                    B = mat(n, 13, 16, 21, p, q, dt) if side == Side.Left else mat(13, n, 16, 21, p, q, dt)
                    Bd = D(B)
                    sl.trmm(side, 2.0, Tv, B)
                    close(D(B), 2.0 * (Tl @ Bd if side == Side.Left else Bd @ Tl))
                    B = mat(B.m(), B.n(), 16, 22, p, q, dt)
                    Bd = D(B)
                    sl.trsm(side, 0.5, Tv, B)
                    X = D(B)
                    close(Tl @ X if side == Side.Left else X @ Tl, 0.5 * Bd, 1e-10)


def check_methods_and_trmm_flops(p, q, dt=torch.float64):
    """trsmA and trsmB (work_trsmA.cc / work_trsm.cc), hemmA and hemmC
    agree with the fp64 oracle on skinny and wide right-hand sides, and the
    distributed trmm multiplies only the stored triangle: the GEMM + TRMM
    flops summed over all ranks equal m^2 n exactly (a dense product would
    be 2 m^2 n)."""
    import torch.distributed as dist
    from slate_amd import ops
    n = 64
    T = mat(n, n, 16, 30, p, q, dt)
    Td = D(T) + 8.0 * torch.eye(n, dtype=dt)
    sl.from_dense(T, Td)
    for uplo in (Uplo.Lower, Uplo.Upper):
        Tl = tri(Td, uplo)
        for nrhs in (9, 40):
            for meth in (MethodTrsm.A, MethodTrsm.B):
                for side in (Side.Left, Side.Right):
                    B = mat(n, nrhs, 16, 31, p, q, dt) if side == Side.Left else mat(nrhs, n, 16, 31, p, q, dt)
                    Bd = D(B)
                    sl.trsm(side, 0.5, sl.TriangularMatrix(uplo, T), B, {Option.MethodTrsm: meth})
                    X = D(B)
                    close(Tl @ X if side == Side.Left else X @ Tl, 0.5 * Bd, 1e-10)
        nrhs = 24
        B = mat(n, nrhs, 16, 32, p, q, dt)
        Bd = D(B)
        with ops.flop_counter() as fc:
            sl.trmm(Side.Left, 1.0, sl.TriangularMatrix(uplo, T), B)
        tot = torch.tensor([fc.flops], dtype=torch.int64)
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(tot)
        assert int(tot) == n * n * nrhs, (int(tot), n * n * nrhs)
        close(D(B), Tl @ Bd)
    for meth in (MethodHemm.A, MethodHemm.C):
        for side in (Side.Left, Side.Right):
            for uplo in (Uplo.Lower, Uplo.Upper):
                for sym in (False, True):
                    cls = sl.SymmetricMatrix if sym else sl.HermitianMatrix
                    A = herm(48, 16, 33, p, q, dt, uplo, cls)
                    Afull = full(D(sl.Matrix(_storage=A.storage)), uplo, not sym)
                    for w in (11, 40):
                        B = mat(48, w, 16, 34, p, q, dt) if side == Side.Left else mat(w, 48, 16, 34, p, q, dt)
                        C = mat(B.m(), B.n(), 16, 35, p, q, dt)
                        Bd, Cd = D(B), D(C)
                        (sl.symm if sym else sl.hemm)(side, 1.5, A, B, 0.5, C, {Option.MethodHemm: meth})
                        close(D(C), 1.5 * (Afull @ Bd if side == Side.Left else Bd @ Afull) + 0.5 * Cd)


ALL = [check_redistribute, check_conj_transpose_keeps_other_triangle, check_potrf_upper_keeps_lower,
       check_gemm_all, check_gemmA, check_rank_k, check_hemm, check_trmm_trsm, check_methods_and_trmm_flops]


def _run(rank, size, p, q, names, complex_too):
    for f in ALL:
        if f.__name__ in names:
            f(p, q)
            if complex_too:
                f(p, q, torch.complex128)


@pytest.mark.parametrize("check", ALL, ids=lambda f: f.__name__)
def test_single_rank(check):
    check(1, 1)
    check(1, 1, torch.complex128)


@pytest.mark.parametrize("grid", [(2, 1), (1, 2)])
def test_two_ranks(grid):
    run_dist(_run, 2, *grid, [f.__name__ for f in ALL], True)


def test_four_ranks():
    run_dist(_run, 4, 2, 2, [f.__name__ for f in ALL], False)


def test_eight_ranks_2x4():
    run_dist(_run, 8, 2, 4, [f.__name__ for f in ALL], False, timeout=900)


def _gather_roots(rank, size, p, q):
    import slate_amd as sl
    from slate_amd.models.aux import allgather_dense
    A = sl.Matrix(37, 29, nb=8, p=p, q=q)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rands", 3)
    ref = allgather_dense(A)
    for root in range(size):
        D = sl.gather(A, root)
        if rank == root:
            assert D is not None and (D.cpu() - ref.cpu()).abs().max() == 0
        else:
            assert D is None


def test_gather_to_root():
    """Matrix::gather: the whole matrix on the root only (piece-level
    redistribution onto rank 0, then one send to another root)."""
    run_dist(_gather_roots, 4, 2, 2)


def _hemmC_workspace(rank, size, p, q):
    import torch
    import slate_amd as sl
    from slate_amd.core.enums import MethodHemm, Option, Side, Uplo
    from slate_amd.models import blas3
    n, nb, w = 96, 8, 40
    for uplo in (Uplo.Lower, Uplo.Upper):
        A = sl.HermitianMatrix(uplo, n, nb=nb, p=p, q=q, dtype=torch.complex128)
        A.insertLocalTiles()
        sl.generate_matrix(A, "rands", 41)
        B = sl.Matrix(n, w, nb=nb, p=p, q=q, dtype=torch.complex128)
        B.insertLocalTiles()
        sl.generate_matrix(B, "rands", 42)
        C = sl.Matrix(n, w, nb=nb, p=p, q=q, dtype=torch.complex128)
        C.insertLocalTiles()
        sl.hemm(Side.Left, 1.0, A, B, 0.0, C, {Option.MethodHemm: MethodHemm.C})
        lb = A.local_block()
        # (local rows + local cols) x nb, never the n x n copy
        bound = (lb.mloc + lb.nloc + C.local_block().nloc) * nb
        assert blas3.HEMMC_STATS["workspace_elems"] <= bound, (blas3.HEMMC_STATS, bound)
        assert blas3.HEMMC_STATS["workspace_elems"] < n * n // (p * q)


def test_hemmC_workspace_2x4():
    """hemmC assembles each block column of the full Hermitian matrix from
    the stored triangle per step (SLATE src/hemmC.cc:147-429): per-rank
    workspace O((local rows + local cols) nb), no n x n materialisation."""
    run_dist(_hemmC_workspace, 8, 2, 4)
