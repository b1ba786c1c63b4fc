"""Python-free native path: libslate_amd_native.so (HIP kernels + C++ runtime,
RCCL / host-staged transports) driven from C++ (examples/cpp/ex_native.cc)
and from C through the ScaLAPACK / BLACS / LAPACK symbols
(examples/c/ex_native_scalapack.c).  The binaries run with an environment
that has no Python library path and do not link libpython.

Multi-rank grids (2x2, 1x4, 2x1) run on ONE GPU through the host-staged
transport (SLATE_AMD_NATIVE_TRANSPORT=host): the p x q drivers, the SUMMA
broadcasts, the distributed LU panel and the tile redistributions execute
exactly as over RCCL, only the bytes travel through the host.
"""
import os
import random
import re
import socket
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "slate_amd", "ex_native")
CEXE = os.path.join(ROOT, "slate_amd", "ex_native_scalapack")
LIB = os.path.join(ROOT, "slate_amd", "libslate_amd_native.so")

# relative-residual bounds per precision suffix
TOL = {"s": 2e-4, "c": 2e-4, "d": 1e-12, "z": 1e-12}


def test_native_library_has_no_python_dependency():
    if not os.path.exists(LIB):
        pytest.skip("libslate_amd_native.so not built")
    out = subprocess.run(["ldd", LIB], capture_output=True, text=True).stdout
    assert "python" not in out.lower(), out
    assert "librccl" in out and "libamdhip64" in out, out
    nm = subprocess.run(["nm", "-D", "--undefined-only", LIB], capture_output=True, text=True).stdout
    assert "Py" not in "".join(l.split()[-1] for l in nm.splitlines() if l.split()), "Python symbols referenced"


def test_native_library_exports_lapack_scalapack_blacs():
    if not os.path.exists(LIB):
        pytest.skip("libslate_amd_native.so not built")
    nm = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    names = {l.split()[-1] for l in nm.splitlines() if l.split()}
    want = ["Cblacs_gridinit", "Cblacs_gridinfo", "blacs_gridinfo_", "numroc_", "descinit_",
            "slate_dgesv", "slate_dgetrf_", "slate_zposv", "slate_sgemm_", "slate_dtrsm_", "slate_dgels",
            "slate_zgels", "slate_dgels_", "slate_dsposv", "slate_dsgesv", "slate_zcposv", "slate_zcgesv"]
    for x in "sdcz":
        want += [f"p{x}potrf_", f"p{x}posv_", f"p{x}getrf_", f"p{x}gesv_", f"p{x}getrs_", f"p{x}gemm_",
                 f"p{x}trsm_", f"p{x}lange_", f"p{x}gels_", f"p{x}syrk_", f"p{x}syr2k_", f"p{x}symm_",
                 f"p{x}trmm_", f"p{x}potri_", f"p{x}getri_", f"p{x}lansy_",
                 f"p{x}lantr_", f"p{x}geadd_", f"p{x}laset_", f"p{x}lacpy_", f"p{x}gecon_", f"p{x}pocon_",
                 f"p{x}trcon_", f"slate_{x}gecon_", f"slate_{x}pocon_", f"slate_{x}trcon_"]
    want += ["pssyevd_", "pdsyevd_", "pcheevd_", "pzheevd_", "pssyev_", "pdsyev_", "pcheev_", "pzheev_",
             "slate_dsyev", "slate_dsyevd", "slate_zheev", "slate_zheevd", "psgesvd_", "pdgesvd_", "pcgesvd_",
             "pzgesvd_", "slate_dgesvd", "slate_zgesvd"]
    want += ["pclanhe_", "pzlanhe_", "pcherk_", "pzherk_", "pcher2k_", "pzher2k_", "pchemm_", "pzhemm_"]
    # the LAPACK-style families that lived only in the
    # CPython-backed ABI, and the mixed-precision ScaLAPACK solvers
    for x in "sdcz":
        want += [f"slate_{x}{w}" for w in ("trmm", "syrk", "syr2k", "symm", "getri", "potri", "lansy", "lantr")]
    for x in "cz":
        want += [f"slate_{x}{w}" for w in ("herk", "her2k", "hemm", "lanhe")]
    for x in "sd":
        want += [f"slate_{x}{w}_" for w in ("trmm", "syrk", "syr2k", "symm", "getri", "potri", "lansy", "lantr")]
    want += ["pdsgesv_", "pzcgesv_"]
    missing = [w for w in want if w not in names]
    assert not missing, missing


def _clean_env(rank=None, size=None, port=None, transport=None):
    env = {k: v for k, v in os.environ.items()
           if not k.startswith("PYTHON") and k not in ("LD_PRELOAD_PYTHON",)}
    env["LD_LIBRARY_PATH"] = "/opt/rocm/lib"          # no Python library directory
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "SLATE_AMD_NATIVE_TRANSPORT", "SLATE_AMD_NATIVE_GRID"):
        env.pop(k, None)
    if rank is not None:
        env.update(RANK=str(rank), WORLD_SIZE=str(size), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SLATE_AMD_NATIVE_TRANSPORT=transport)
    return env


def _free_port_block(n):
    """a MASTER_PORT whose next n + 2 ports are free (the host transport
    listens on MASTER_PORT + 2 + rank)"""
    for _ in range(50):
        base = random.randint(20000, 50000)
        ok = True
        for pt in range(base, base + n + 3):
            with socket.socket() as s:
                try:
                    s.bind(("127.0.0.1", pt))
                except OSError:
                    ok = False
                    break
        if ok:
            return base
    raise RuntimeError("no free port block")


def _run_ranks(exe, args, nranks, timeout=240):
    port = _free_port_block(nranks)
    procs = [subprocess.Popen([exe] + args, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                              env=_clean_env(r, nranks, port, "host"))
             for r in range(nranks)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append((p.returncode, out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return outs


def _checks(out):
    return dict(re.findall(r"^check (\S+) (\S+)$", out, re.M))


def _assert_checks(checks, out):
    names = [f"{w}_{x}" for x in "sdcz" for w in ("potrf", "potrs", "gesv", "getrs_conjtrans", "getrf_rect",
                                                   "gemm", "gemm_ct", "norm_max", "norm_fro", "norm_one",
                                                   "trsm_lc", "gels", "herk", "her2k_upper", "syrk",
                                                   "syr2k_upper", "hemm_left", "symm_right", "trmm_luc",
                                                   "potri", "getri", "norm_herm_one", "norm_sym_one",
                                                   "norm_tri_fro", "heev", "heev_orth", "heev_values",
                                                   "gecondest", "svd", "svd_orth", "svd_wide", "svd_wide_orth", "geqrf", "geqrf_wide", "gels_grid",
                                                   "trsm_lt", "trsm_rn", "trsm_rc", "trtri", "trtrm", "gesv_nopiv",
                                                   "cholqr", "cholqr_orth", "gelqf", "sub_potrf", "from_device_potrs", "lu_xchg_bound",
                                                   "svd_values", "gesv_rbt", "hegv1", "hegv2_upper", "hegv3",
                                                   "view_gemm", "view_dims", "view_norm", "view_rejected",
                                                   "tri_view_uplo", "tri_view_trsm", "trapezoid_norm",
                                                   "slice_roundtrip", "empty_like", "sym_syrk_symm",
                                                   "pbsv", "pbsv_upper", "gbmm", "gbsv", "hbmm_left", "hbmm_right",
                                                   "tbsm_upper_conj", "getrf_tntpiv", "tntpiv_growth", "hesv",
                                                   "redistribute")]
    for name in names:
        assert name in checks, (name, out)
        assert float(checks[name]) < TOL[name[-1]], (name, checks[name])
    for name in [f"{w}_{x}" for x in "dz" for w in ("posv_mixed", "gesv_mixed", "posv_gmres", "gesv_gmres")]:
        assert name in checks, (name, out)
        assert float(checks[name]) < TOL[name[-1]], (name, checks[name])
    for name in ("capi_dgesv", "capi_zposv", "capi_dgemm_tn"):
        assert name in checks, (name, out)
        assert float(checks[name]) < 1e-12, (name, checks[name])


@pytest.mark.gpu
def test_native_example_runs_without_python():
    assert os.path.exists(EXE), "slate_amd/ex_native not built (run __graft_entry__.build())"
    ldd = subprocess.run(["ldd", EXE], capture_output=True, text=True, env=_clean_env()).stdout
    assert "python" not in ldd.lower(), ldd
    r = subprocess.run([EXE, "1x1", "8192"], capture_output=True, text=True, env=_clean_env(), timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    _assert_checks(_checks(r.stdout), r.stdout)
    times = re.findall(r"^time potrf n=8192 (\S+) ms (\S+) TF/s info=0$", r.stdout, re.M)
    assert len(times) == 3, r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("grid", ["2x2", "1x4", "2x1"])
def test_native_example_grids_host_transport(grid):
    """p x q grids on one GPU: several ranks share the device through the
    host-staged transport; every check of every precision must pass."""
    p, q = map(int, grid.split("x"))
    outs = _run_ranks(EXE, [grid], p * q)
    for rc, out in outs:
        assert rc == 0, out
    out0 = outs[0][1]
    print(out0)
    assert f"transport host ranks {p * q} grid {grid}" in out0
    checks = _checks(out0)
    _assert_checks(checks, out0)
    # the distributed heev (no n x n on any rank) against the gather path
    for x in "sdcz":
        name = f"heev_grid_vs_gather_{x}"
        assert name in checks, (name, out0)
        assert float(checks[name]) < TOL[x], (name, checks[name])


LEXE = os.path.join(ROOT, "slate_amd", "ex_native_lapack")


@pytest.mark.gpu
@pytest.mark.parametrize("nranks", [1, 2])
def test_native_lapack_more_from_c(nranks):
    """slate_?trmm/syrk/syr2k/symm/getri/potri/lansy/lantr and the complex
    herk/her2k/hemm/lanhe of libslate_amd_native.so, from plain C against
    naive host loops (1 rank, and 2 ranks over the host transport)."""
    assert os.path.exists(LEXE), "slate_amd/ex_native_lapack not built"
    ldd = subprocess.run(["ldd", LEXE], capture_output=True, text=True, env=_clean_env()).stdout
    assert "python" not in ldd.lower(), ldd
    if nranks == 1:
        r = subprocess.run([LEXE, "200"], capture_output=True, text=True, env=_clean_env(), timeout=240)
        outs = [(r.returncode, r.stdout + r.stderr)]
    else:
        outs = _run_ranks(LEXE, ["150"], nranks)
    for rc, out in outs:
        print(out)
        assert rc == 0 and "all checks passed" in out, out
        assert len(_checks(out)) >= 20, out


HEXE = os.path.join(ROOT, "slate_amd", "ex_native_handles")
CPPEXE = os.path.join(ROOT, "slate_amd", "ex_cpp_api_native")


@pytest.mark.gpu
@pytest.mark.parametrize("grid", ["1x1", "2x2"])
def test_cpp_header_api_over_native(grid):
    """The header-only C++ API (include/slate_amd/slate_amd.hh) linked
    against libslate_amd_native.so instead of the deprecated CPython-backed
    libslate_amd_c.so: posv / gesv / getri / trmm / trsm / herk / gels /
    heev / svd_vals / gesv_mixed with sub-matrix and transposed views."""
    assert os.path.exists(CPPEXE), "slate_amd/ex_cpp_api_native not built"
    ldd = subprocess.run(["ldd", CPPEXE], capture_output=True, text=True, env=_clean_env()).stdout
    assert "python" not in ldd.lower() and "libslate_amd_c" not in ldd, ldd
    p, q = map(int, grid.split("x"))
    if p * q == 1:
        r = subprocess.run([CPPEXE, grid], capture_output=True, text=True, env=_clean_env(), timeout=240)
        outs = [(r.returncode, r.stdout + r.stderr)]
    else:
        outs = _run_ranks(CPPEXE, [grid], p * q)
    for rc, out in outs:
        print(out)
        assert rc == 0, out
        lines = [ln for ln in out.splitlines() if ln.startswith("rank ") and "iterations" not in ln]
        assert len(lines) == 9, out
        for ln in lines:
            assert "FAILED" not in ln, ln
            assert float(ln.split()[-1]) < 1e-10, ln


@pytest.mark.gpu
def test_native_trace_chrome_json(tmp_path):
    """Native tracing (SLATE Trace): a traced dpotrf + dgetrf on a 2 x 2 grid
    (host transport) gathers every rank's host and per-stream device spans
    to rank 0, which writes one Chrome trace-event JSON; timers() reports the
    phases (host and @device seconds)."""
    import json
    path = str(tmp_path / "native_trace.json")
    port = _free_port_block(4)
    procs = []
    for r in range(4):
        env = _clean_env(r, 4, port, "host")
        env["EX_NATIVE_TRACE"] = path
        procs.append(subprocess.Popen([EXE, "2x2"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                                      env=env))
    outs = [p.communicate(timeout=240)[0] for p in procs]
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out
    print(outs[0])
    ev = json.load(open(path))["traceEvents"]
    spans = [e for e in ev if e.get("ph") == "X"]
    assert {e["pid"] for e in spans} == {0, 1, 2, 3}
    names = {e["name"] for e in spans}
    for nm in ("potrf", "potrf::panel", "potrf::bcast", "potrf::lookahead", "potrf::update", "getrf",
               "getrf::panel", "getrf::update"):
        assert nm in names, (nm, sorted(names))
    # device spans sit on the stream tracks (tid 1 panel, 2 update, 3 comm)
    tids = {(e["name"], e["tid"]) for e in spans}
    assert ("potrf::panel", 1) in tids and ("potrf::update", 2) in tids and ("potrf::bcast", 3) in tids, tids
    assert all(e["dur"] >= 0 for e in spans)
    timers = dict(re.findall(r"^timer (\S+) (\S+)$", outs[0], re.M))
    assert float(timers["potrf"]) > 0 and float(timers["potrf::update@device"]) > 0, timers


@pytest.mark.gpu
@pytest.mark.parametrize("grid", ["1x1", "2x2"])
def test_native_handle_capi_from_c(grid):
    """The opaque-handle C API (slate_amd_matrix_create, _posv, _gesv,
    _gemm on transposed views, _unmqr left / right, _heev, _hegv, mixed /
    GMRES / RBT solvers, ...) served by libslate_amd_native.so: no Python in
    the process (the CPython-embedding libslate_amd_c.so is deprecated)."""
    assert os.path.exists(HEXE), "slate_amd/ex_native_handles not built"
    ldd = subprocess.run(["ldd", HEXE], capture_output=True, text=True, env=_clean_env()).stdout
    assert "python" not in ldd.lower() and "libslate_amd_c" not in ldd, ldd
    p, q = map(int, grid.split("x"))
    if p * q == 1:
        r = subprocess.run([HEXE, grid], capture_output=True, text=True, env=_clean_env(), timeout=240)
        outs = [(r.returncode, r.stdout + r.stderr)]
    else:
        outs = _run_ranks(HEXE, [grid], p * q)
    for rc, out in outs:
        print(out)
        assert rc == 0, out
    out0 = outs[0][1]
    assert "all checks passed" in out0, out0
    assert len(_checks(out0)) >= 25, out0


@pytest.mark.gpu
@pytest.mark.parametrize("grid", ["1x1", "2x2", "2x1"])
def test_native_scalapack_from_c_without_python(grid):
    """pdpotrf_/pdgesv_/pdgetrf_/pzgesv_/pdgemm_/pdlange_ and slate_dgetrf_
    called from plain C on local block-cyclic arrays."""
    assert os.path.exists(CEXE), "slate_amd/ex_native_scalapack not built"
    ldd = subprocess.run(["ldd", CEXE], capture_output=True, text=True, env=_clean_env()).stdout
    assert "python" not in ldd.lower(), ldd
    p, q = map(int, grid.split("x"))
    if p * q == 1:
        r = subprocess.run([CEXE, grid], capture_output=True, text=True, env=_clean_env(), timeout=240)
        outs = [(r.returncode, r.stdout + r.stderr)]
    else:
        outs = _run_ranks(CEXE, [grid], p * q)
    names = ("pdpotrs", "pdpotrs_upper", "pdgesv", "pdgetrs", "pdlange_fro", "pdgemm_tn", "pdsyrk_lower", "pdtrmm_lun", "pdpotri", "pdgetri", "pdlaset_lacpy_geadd",
             "pzgesv", "slate_dgetrf_", "pdgemm_sub", "pdpotrs_sub", "pdgetrs_sub", "pdtrsm_right", "pztrsm_trans",
             "pdgecon", "pdpocon", "pdtrcon", "pdsyevd", "pdgesvd", "pdgels", "pdsgesv")
    for rank, (rc, out) in enumerate(outs):
        print(out)
        assert rc == 0, out
        found = dict(re.findall(rf"^check r{rank} (\S+) (\S+)$", out, re.M))
        for nm in names:
            assert nm in found, (nm, out)
            assert float(found[nm]) < 1e-11, (nm, found[nm], out)
