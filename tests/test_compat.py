"""LAPACK / ScaLAPACK-style front-ends (reference: lapack_api/ and
scalapack_api/ smoke tests run the interposed routines against the
reference library; here against PyTorch fp64)."""
import numpy as np
import pytest
import torch

from slate_amd.compat import lapack as L
from slate_amd.compat import scalapack as S

from dist_util import run_dist


def _spd(n, seed, dt=np.float64):
    r = np.random.default_rng(seed)
    X = r.standard_normal((n, n))
    if np.dtype(dt).kind == 'c':
        X = X + 1j * r.standard_normal((n, n))
    return (X @ X.conj().T + n * np.eye(n)).astype(dt)


def test_lapack_potrf_posv_gesv():
    n = 70
    A = np.asfortranarray(_spd(n, 1))
    B = np.asfortranarray(np.random.default_rng(2).standard_normal((n, 3)))
    A0, B0 = A.copy(), B.copy()
    assert L.dposv('L', n, 3, A, n, B, n) == 0
    assert np.abs(A0 @ B - B0).max() < 1e-10
    M = np.asfortranarray(np.random.default_rng(3).standard_normal((n, n)))
    M0 = M.copy()
    B = B0.copy(order='F')
    ipiv = np.zeros(n, dtype=np.int64)
    assert L.dgesv(n, 3, M, n, ipiv, B, n) == 0
    assert np.abs(M0 @ B - B0).max() < 1e-10
    assert ipiv.min() >= 1


def test_lapack_flat_storage_and_complex():
    n, lda = 40, 45
    A = _spd(n, 4, np.complex128)
    flat = np.zeros(lda * n, dtype=np.complex128)
    for j in range(n):
        flat[j * lda:j * lda + n] = A[:, j]
    assert L.zpotrf('L', n, flat, lda) == 0
    Lf = np.tril(np.stack([flat[j * lda:j * lda + n] for j in range(n)], axis=1))
    assert np.abs(Lf @ Lf.conj().T - A).max() < 1e-10


def test_lapack_gemm_trsm_geqrf_gels_syev_gesvd():
    r = np.random.default_rng(5)
    m, n, k = 30, 20, 10
    A, B, C = (np.asfortranarray(r.standard_normal(s)) for s in ((m, k), (k, n), (m, n)))
    C0 = C.copy()
    L.dgemm('N', 'N', m, n, k, 2.0, A, m, B, k, 0.5, C, m)
    assert np.abs(C - (2 * A @ B + 0.5 * C0)).max() < 1e-12
    T = np.asfortranarray(np.tril(r.standard_normal((n, n))) + n * np.eye(n))
    X = np.asfortranarray(r.standard_normal((n, 4)))
    X0 = X.copy()
    L.dtrsm('L', 'L', 'N', 'N', n, 4, 1.0, T, n, X, n)
    assert np.abs(T @ X - X0).max() < 1e-12
    G = np.asfortranarray(r.standard_normal((m, n)))
    G0 = G.copy()
    Bg = np.asfortranarray(r.standard_normal((m, 2)))
    Bg0 = Bg.copy()
    L.dgels('N', m, n, 2, G, m, Bg, m)
    assert np.abs(Bg[:n] - np.linalg.lstsq(G0, Bg0, rcond=None)[0]).max() < 1e-10
    H = np.asfortranarray(_spd(25, 6) - 30 * np.eye(25))
    H0 = H.copy()
    w = np.zeros(25)
    L.dsyev('V', 'L', 25, H, 25, w)
    assert np.abs(w - np.linalg.eigvalsh(H0)).max() < 1e-10
    assert np.abs(H0 @ H - H * w).max() < 1e-10
    Sg = np.asfortranarray(r.standard_normal((m, n)))
    Sg0 = Sg.copy()
    s = np.zeros(n)
    U = np.zeros((m, n), order='F')
    VT = np.zeros((n, n), order='F')
    L.dgesvd('S', 'S', m, n, Sg, m, s, U, m, VT, n)
    assert np.abs(U @ np.diag(s) @ VT - Sg0).max() < 1e-10
    assert abs(L.dlange('F', m, n, Sg0, m) - np.linalg.norm(Sg0)) < 1e-10


def _local(Aglob, nb, p, q, pr, pc):
    m, n = Aglob.shape
    rows = [i for i in range(m) if (i // nb) % p == pr]
    cols = [j for j in range(n) if (j // nb) % q == pc]
    return np.asfortranarray(Aglob[np.ix_(rows, cols)]), rows, cols


def _sca(rank, size, p, q):
    ctxt = S.blacs_gridinit(p, q)
    _, _, pr, pc = S.blacs_gridinfo(ctxt)
    n, nb = 60, 16
    A = _spd(n, 7)
    B = np.random.default_rng(8).standard_normal((n, 2))
    Al, _, _ = _local(A, nb, p, q, pr, pc)
    Bl, rows, cols = _local(B, nb, p, q, pr, pc)
    desca = [1, ctxt, n, n, nb, nb, 0, 0, max(1, Al.shape[0])]
    descb = [1, ctxt, n, 2, nb, nb, 0, 0, max(1, Bl.shape[0])]
    assert S.pdposv('L', n, 2, Al, 1, 1, desca, Bl, 1, 1, descb) == 0
    X = np.linalg.solve(A, B)
    if Bl.size:
        assert np.abs(Bl - X[np.ix_(rows, cols)]).max() < 1e-10
    M = np.random.default_rng(9).standard_normal((n, n))
    Ml, _, _ = _local(M, nb, p, q, pr, pc)
    Bl, rows, cols = _local(B, nb, p, q, pr, pc)
    ipiv = np.zeros(n, dtype=np.int64)
    assert S.pdgesv(n, 2, Ml, 1, 1, desca, ipiv, Bl, 1, 1, descb) == 0
    X = np.linalg.solve(M, B)
    if Bl.size:
        assert np.abs(Bl - X[np.ix_(rows, cols)]).max() < 1e-10


@pytest.mark.parametrize("grid", [(2, 1), (1, 2)])
def test_scalapack_grid(grid):
    run_dist(_sca, 2, *grid)


def test_c_api(tmp_path):
    """Compile and run the C example against libslate_amd_c.so."""
    import os
    import subprocess
    import sysconfig
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "slate_amd")
    exe = str(tmp_path / "ex_capi")
    libdir = sysconfig.get_config_var("LIBDIR")
    cmd = ["gcc", "-O1", os.path.join(root, "examples", "c", "ex_capi.c"), "-I", os.path.join(root, "include"),
           "-L", lib, "-lslate_amd_c", "-Wl,-rpath," + lib, "-L", libdir,
           "-l" + "python" + sysconfig.get_config_var("LDVERSION"), "-lm", "-o", exe]
    subprocess.run(cmd, check=True)
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""),
               SLATE_AMD_LAPACK_TARGET="host")
    r = subprocess.run([exe], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    assert "dgesv info=0" in r.stdout


def test_fortran_module(tmp_path):
    """Compile the Fortran module (include/slate_amd/slate_amd.f90) and the
    Fortran example with flang, link against libslate_amd_c.so and run it."""
    import os
    import shutil
    import subprocess
    import sysconfig
    flang = shutil.which("flang") or ("/opt/rocm/llvm/bin/flang" if os.path.exists("/opt/rocm/llvm/bin/flang") else None)
    if flang is None:
        pytest.skip("no Fortran compiler")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "slate_amd")
    exe = str(tmp_path / "ex_fortran")
    cmd = [flang, "-O1", "-J", str(tmp_path), os.path.join(root, "include", "slate_amd", "slate_amd.f90"),
           os.path.join(root, "examples", "fortran", "ex_fortran.f90"), "-L", lib, "-lslate_amd_c",
           "-Wl,-rpath," + lib, "-L", sysconfig.get_config_var("LIBDIR"),
           "-lpython" + sysconfig.get_config_var("LDVERSION"), "-o", exe]
    subprocess.run(cmd, check=True, cwd=str(tmp_path))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""),
               SLATE_AMD_LAPACK_TARGET="host")
    r = subprocess.run([exe], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    assert "dgesv info=0" in r.stdout and "dposv info=0" in r.stdout


def _build_c(tmp_path, src, name):
    import os
    import subprocess
    import sysconfig
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "slate_amd")
    exe = str(tmp_path / name)
    cxx = src.endswith(".cc")
    cmd = (["g++", "-std=c++17", "-O1", os.path.join(root, "examples", "cpp", src)] if cxx else
           ["gcc", "-O1", os.path.join(root, "examples", "c", src)]) + ["-I", os.path.join(root, "include"),
           "-L", lib, "-lslate_amd_c", "-Wl,-rpath," + lib, "-L", sysconfig.get_config_var("LIBDIR"),
           "-lpython" + sysconfig.get_config_var("LDVERSION"), "-lm", "-o", exe]
    subprocess.run(cmd, check=True)
    return exe, root


@pytest.mark.parametrize("grid", ["1x1", "1x2", "2x1"])
def test_c_scalapack_and_handles(tmp_path, grid):
    """pdposv_/pdgesv_ on sub-matrices starting inside a tile, pdgemm_, the
    minimal BLACS and the handle API -- from C, one process per rank."""
    import os
    import subprocess
    from dist_util import _free_port
    exe, root = _build_c(tmp_path, "ex_scalapack.c", "ex_scalapack")
    p, q = map(int, grid.split("x"))
    size = p * q
    port = str(_free_port())
    procs = []
    for r in range(size):
        env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""),
                   SLATE_AMD_SCALAPACK_TARGET="host", OMP_NUM_THREADS="2")
        if size > 1:
            env.update(RANK=str(r), WORLD_SIZE=str(size), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=port)
        procs.append(subprocess.Popen([exe, grid], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = [pr.communicate(timeout=300)[0] for pr in procs]
    for pr, out in zip(procs, outs):
        assert pr.returncode == 0, out
        lines = [ln for ln in out.splitlines() if ln.startswith("rank ")]
        assert len(lines) == 4, out
        for ln in lines:
            assert "info=0" in ln or "pdgemm" in ln, ln
            val = float(ln.split("=")[-1])
            assert val < 1e-9, ln


@pytest.mark.parametrize("grid", ["1x1", "2x1"])
def test_c_compat_more(tmp_path, grid):
    """Round-3 LAPACK-style (trmm/syrk/symm/getri/gecon/lansy/lantr/syevd/
    dsgesv/zherk/zlanhe) and ScaLAPACK (pdtrmm/pdsymm/pdsyrk/pdgetri/pdgecon/
    pdpotri/pdlansy/pdsyev/pdsyevd/pdsgesv) entry points, from C."""
    import os
    import subprocess
    from dist_util import _free_port
    exe, root = _build_c(tmp_path, "ex_compat_more.c", "ex_compat_more")
    p, q = map(int, grid.split("x"))
    size = p * q
    port = str(_free_port())
    procs = []
    for r in range(size):
        env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""),
                   SLATE_AMD_SCALAPACK_TARGET="host", SLATE_AMD_LAPACK_TARGET="host", OMP_NUM_THREADS="2")
        if size > 1:
            env.update(RANK=str(r), WORLD_SIZE=str(size), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=port)
        procs.append(subprocess.Popen([exe, grid], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = [pr.communicate(timeout=600)[0] for pr in procs]
    for r, (pr, out) in enumerate(zip(procs, outs)):
        assert pr.returncode == 0, out
        lines = [ln for ln in out.splitlines() if ln.startswith("rank ")]
        assert len(lines) == (20 if r == 0 else 9), out
        for ln in lines:
            assert "FAILED" not in ln, ln
            if "info=" in ln:
                assert "info=0" in ln, ln
            else:
                assert float(ln.split()[-1]) < 1e-9, ln


@pytest.mark.parametrize("grid", ["1x1", "1x2", "2x1"])
def test_cpp_api(tmp_path, grid):
    """The C++ API (include/slate_amd/slate_amd.hh): posv/gesv/getri/trmm/
    trsm/herk/gels/heev/svd_vals/gesv_mixed with sub-matrix and
    conjugate-transposed views and options, one process per rank; every
    residual is computed by library routines."""
    import os
    import subprocess
    from dist_util import _free_port
    exe, root = _build_c(tmp_path, "ex_cpp_api.cc", "ex_cpp_api")
    p, q = map(int, grid.split("x"))
    size = p * q
    port = str(_free_port())
    procs = []
    for r in range(size):
        env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""), OMP_NUM_THREADS="2")
        if size > 1:
            env.update(RANK=str(r), WORLD_SIZE=str(size), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=port)
        procs.append(subprocess.Popen([exe, grid], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = [pr.communicate(timeout=600)[0] for pr in procs]
    for pr, out in zip(procs, outs):
        assert pr.returncode == 0, out
        lines = [ln for ln in out.splitlines() if ln.startswith("rank ") and "iterations" not in ln]
        assert len(lines) == 9, out
        for ln in lines:
            assert "FAILED" not in ln, ln
            assert float(ln.split()[-1]) < 1e-10, ln


def test_lapack_upper_potrf_potri_keep_other_triangle():
    """LAPACK never touches the unreferenced triangle: after potrf('U') /
    potri('U') the strictly-lower part is exactly what the caller left."""
    import numpy as np
    from slate_amd.compat import lapack
    n = 7
    g = np.random.default_rng(1)
    M = g.standard_normal((n, n))
    A = np.asfortranarray(M @ M.T + n * np.eye(n))
    S = A.copy()
    A[np.tril_indices(n, -1)] = 77.0
    assert lapack.dpotrf('U', n, A, n) == 0
    assert np.all(A[np.tril_indices(n, -1)] == 77.0)
    R = np.triu(A)
    assert np.abs(R.T @ R - S).max() < 1e-12 * np.abs(S).max() * n
    assert lapack.dpotri('U', n, A, n) == 0
    assert np.all(A[np.tril_indices(n, -1)] == 77.0)
