"""Matrix generator (`slate_matgen`: include/slate/generate_matrix.hh:17-75,
matgen/random.cc:36-60, matgen/generate_matrix_utils.cc).

Entries are a pure function of (seed, global i, global j) via a
counter-based Philox4x32-10 stream shared by the host runtime and the gfx950
kernel, so the same matrix is produced for any grid / tile size / device,
and a rank fills its local buffer on the GPU without host staging.
"""
from __future__ import annotations

from .. import ops
from ..core.exceptions import SlateError
from ..core.storage import DEV

KINDS = {
    "zeros": 0, "zero": 0, "ones": 1, "identity": 2, "ij": 3, "jordan": 4,
    "rand": 10, "rands": 11, "randn": 12, "randb": 13, "randr": 14,
    "rand_dominant": 20, "diag_dominant": 20, "rands_dominant": 20, "hpd": 21,
    "rands_hermitian": 22,
    "minij": 30, "hilb": 31, "lehmer": 32, "frank": 33, "moler": 34,
    "jordant": 40, "chebspec": 41, "circul": 42, "fiedler": 43, "gfpp": 44, "kms": 45, "orthog": 46,
    "riemann": 47, "ris": 48, "zielkens": 49, "lotkin": 50, "redheff": 51, "triw": 52, "pei": 53,
    "tridiag": 54, "toeppen": 55, "parter": 56, "cauchy": 57, "chow": 58, "clement": 59, "gcdmat": 60,
}
# kinds built from a spectrum (SLATE generate_matrix_utils.cc: diag, svd,
# poev/spd, heev/syev; geev/geevx are "not yet implemented" there too)
SPECTRAL = {"diag", "svd", "poev", "spd", "heev", "syev"}
DISTS = {"logrand", "arith", "geo", "cluster0", "cluster1", "rarith", "rgeo", "rcluster0", "rcluster1",
         "specified", "rand", "rands", "randn"}


class MatgenParams:
    """SLATE MatgenParams: kind (with _dist / _scaling / _modifier suffixes),
    seed, scale, cond (default 1/sqrt(eps)), condD (column scaling
    condition, default 1), sigma (the spectrum for _specified)."""

    def __init__(self, kind="rands", seed=42, scale=1.0, cond=None, condD=None, sigma=None):
        self.kind, self.seed, self.scale = kind, seed, scale
        self.cond, self.condD, self.sigma = cond, condD, sigma


def _decode(kind):
    """base, dist, scaling, dominant, zero_col spec (SLATE decode_matrix)."""
    toks = [t for t in str(kind).replace("-", "_").split("_") if t]
    if not toks:
        raise SlateError("empty matrix kind")
    base = toks[0].lower()
    dist, scal, dominant, zcol = None, None, False, None
    for t in toks[1:]:
        tl = t.lower()
        if tl in DISTS and base in SPECTRAL:
            dist = tl
        elif tl in ("ufl", "ofl", "small", "large"):
            scal = tl
        elif tl == "dominant":
            dominant = True
        elif tl.startswith("zerocol"):
            zcol = tl[7:]
        elif tl == "hermitian" and base == "rands":
            base = "rands_hermitian"
        else:
            raise SlateError(f"unknown matrix kind suffix {t!r} in {kind!r}")
    return base, dist, scal, dominant, zcol


def _real_eps_min(dtype):
    import torch
    f = torch.finfo(torch.float32 if dtype in (torch.float32, torch.complex64) else torch.float64)
    return f.eps, f.tiny


def sigma_values(dist, n, cond, seed, dtype=None, specified=None):
    """The spectrum of a spectral kind (descending magnitudes for the
    deterministic distributions): SLATE generate_sigma."""
    import math
    import torch
    g = torch.Generator().manual_seed(int(seed) * 7919 + 17)
    dist = dist or "logrand"
    i = torch.arange(n, dtype=torch.float64)
    den = max(n - 1, 1)
    if dist == "specified":
        if specified is None:
            raise SlateError("_specified needs sigma")
        return torch.as_tensor(specified, dtype=torch.float64)[:n].clone()
    if dist in ("arith", "rarith"):
        s = 1 - i / den * (1 - 1 / cond)
    elif dist in ("geo", "rgeo"):
        s = cond ** (-i / den)
    elif dist in ("cluster0", "rcluster0"):
        s = torch.full((n,), 1 / cond, dtype=torch.float64)
        if n:
            s[0] = 1
    elif dist in ("cluster1", "rcluster1"):
        s = torch.ones(n, dtype=torch.float64)
        if n:
            s[-1] = 1 / cond
    elif dist == "logrand":
        s = torch.exp(torch.rand(n, generator=g, dtype=torch.float64) * math.log(1 / cond))
    elif dist == "rand":
        s = torch.rand(n, generator=g, dtype=torch.float64)
    elif dist == "rands":
        s = torch.rand(n, generator=g, dtype=torch.float64) * 2 - 1
    else:
        s = torch.randn(n, generator=g, dtype=torch.float64)
    if dist.startswith("r") and dist not in ("rand", "rands", "randn"):
        s = s.flip(0)
    return s


def _set_diag(A, vals, add=False):
    """A(i, i) = vals[i] (or += when add) on this rank's local diagonal
    entries (vals replicated on the host)."""
    import torch
    s = A.storage
    k = min(A.m(), A.n())
    if s.bc is None:
        for (i, j, slot) in list(s.tiles.keys()):
            if i != j or not s.tileIsLocal(i, j):
                continue
            t = s.tiles[(i, j, slot)]
            r0 = s.row_offsets[i]
            w = min(t.shape[0], t.shape[1], k - r0)
            if w > 0:
                d = t.diagonal()[:w]
                v = vals[r0:r0 + w].to(d.dtype).to(d.device)
                d.add_(v) if add else d.copy_(v)
        return
    lb = A.local_block()
    if lb.mloc == 0 or lb.nloc == 0:
        return
    rows = {lb.global_row(i): i for i in range(lb.mloc)}
    pairs = [(rows[g], j, g) for j in range(lb.nloc) for g in (lb.global_col(j),) if g in rows and g < k]
    if not pairs:
        return
    dev = lb.data.device
    li = torch.as_tensor([p[0] for p in pairs], device=dev)
    lj = torch.as_tensor([p[1] for p in pairs], device=dev)
    v = vals[torch.as_tensor([p[2] for p in pairs])].to(lb.data.dtype).to(dev)
    if add:
        lb.data[li, lj] += v
    else:
        lb.data[li, lj] = v
    s.mark_local_modified(s.origin_slot)


def _random_unitary_apply(A, side, seed, k):
    """A := Q A (side 'L') or A Q^H ('R') with Q the random unitary of a QR
    of a randn matrix (distributed geqrf + unmqr, no dense gather)."""
    from ..core.matrix import Matrix, TriangularFactors
    from ..core.enums import Op, Side
    from ..models.qr import geqrf, unmqr
    s = A.storage
    bc = s.bc
    mm = A.m() if side == 'L' else A.n()
    X = Matrix(mm, k, nb=bc.nb, p=bc.p, q=bc.q, comm=s.comm, dtype=s.dtype, device=s.device, order=bc.order)
    X.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    generate_matrix(X, "randn", seed)
    T = TriangularFactors()
    geqrf(X, T)
    if side == 'L':
        unmqr(Side.Left, Op.NoTrans, X, T, A)
    else:
        unmqr(Side.Right, Op.ConjTrans, X, T, A)


def _zero_col(A, spec, herm):
    from ..models.aux import set as aset
    n = A.n()
    c = int(round(float(spec) * (n - 1))) if "." in spec else int(spec)
    if not 0 <= c < n:
        raise SlateError(f"zerocol {c} out of range")
    aset(0.0, 0.0, A.slice(0, A.m() - 1, c, c))
    if herm:
        aset(0.0, 0.0, A.slice(c, c, 0, n - 1))


def generate_matrix(A, kind="rands", seed=42, scale=1.0, cond=None, condD=None, sigma=None):
    """Fill A (any view of a block-cyclic or per-tile matrix) with a test
    matrix (SLATE generate_matrix, matgen/generate_matrix_ge.cc):

    * elementwise kinds from the shared Philox / closed-form generator
      (zeros ones identity ij jordan jordanT rand rands randn randb randr,
      Matlab gallery: minij hilb lehmer frank moler chebspec circul fiedler
      gfpp kms orthog riemann ris zielkeNS lotkin redheff triw pei tridiag
      toeppen parter cauchy chow clement gcdmat; rand_dominant, hpd);
    * spectral kinds diag / svd / poev (spd) / heev (syev) with a
      distribution suffix (_logrand default, _arith _geo _cluster0
      _cluster1, reversed _r..., _rand _rands _randn, _specified) and
      condition number ``cond`` (default 1/sqrt(eps)): A = Sigma,
      U Sigma V^H, V Sigma V^H with random unitary U, V applied by the
      distributed QR (geqrf + unmqr) -- heev flips random signs;
    * scaling suffixes _ufl _ofl _small _large; modifiers _dominant and
      _zerocolN / _zerocolFRAC.  Returns the spectrum for spectral kinds."""
    if isinstance(kind, MatgenParams):
        kind, seed, scale, cond, condD, sigma = kind.kind, kind.seed, kind.scale, kind.cond, kind.condD, kind.sigma
    s = A.storage
    base, dist, scal, dominant, zcol = _decode(kind)
    eps, tiny = _real_eps_min(s.dtype)
    sc = {"ufl": tiny, "ofl": 1 / tiny, "small": tiny ** 0.5, "large": (1 / tiny) ** 0.5}.get(scal, 1.0)
    herm = getattr(A, "_kind", "general") in ("hermitian", "symmetric")
    out = None
    if base in ("poev", "spd", "heev", "syev") and dist is None and cond is None and sigma is None:
        # no spectrum requested: the O(n^2) elementwise variants (Hermitian
        # rands + max(m, n) I for poev/spd -- HPD by diagonal dominance --
        # and Hermitian rands for heev), used by the benchmarks
        base = "hpd" if base in ("poev", "spd") else "rands_hermitian"
    if base in SPECTRAL:
        out = _generate_spectral(A, base, dist, cond if cond is not None else 1 / eps ** 0.5, seed, sigma,
                                 scale * sc)
        if condD is not None and condD != 1:
            # column scaling A D, D geometric with condition condD
            import torch
            from ..models.aux import scale_row_col
            n = A.n()
            d = condD ** (-torch.arange(n, dtype=torch.float64) / max(n - 1, 1))
            scale_row_col('C', None, d, A)
    else:
        k = KINDS.get(base.lower())
        if k is None:
            raise SlateError(f"unknown matrix kind {kind!r}")
        _fill(A, k, seed, scale * sc)
        if dominant and k not in (20, 21):
            import torch
            _set_diag(A, torch.full((min(A.m(), A.n()),), float(max(A.m(), A.n())) * scale * sc,
                                    dtype=torch.float64), add=True)
    if zcol is not None:
        _zero_col(A, zcol, herm)
    return out if out is not None else A


def _generate_spectral(A, base, dist, cond, seed, sigma, scale):
    import torch
    from ..models.aux import set as aset
    s = A.storage
    if s.bc is None:
        raise SlateError(f"matrix kind {base!r} needs a block-cyclic matrix")
    m, n = A.m(), A.n()
    k = min(m, n)
    if base in ("poev", "spd", "heev", "syev") and m != n:
        raise SlateError(f"{base}: square matrix required")
    sv = sigma_values(dist, k, cond, seed, s.dtype, sigma) * scale
    if base == "heev" or base == "syev":
        g = torch.Generator().manual_seed(int(seed) + 1)
        sgn = torch.where(torch.rand(k, generator=g) < 0.5, -1.0, 1.0).to(torch.float64)
        sv = sv * sgn
    if base in ("poev", "spd"):
        sv = sv.abs()
    # Hermitian storage: build the full matrix in a general twin, copy the triangle
    target = A
    if getattr(A, "_kind", "general") != "general":
        from ..core.matrix import Matrix
        bc = s.bc
        target = Matrix(m, n, nb=bc.nb, p=bc.p, q=bc.q, comm=s.comm, dtype=s.dtype, device=s.device,
                        order=bc.order)
        target.insertLocalTiles(device=s.device.index if s.device.type == "cuda" else -1)
    aset(0.0, 0.0, target)
    _set_diag(target, sv)
    if base != "diag":
        _random_unitary_apply(target, 'L', seed + 101, k)
        _random_unitary_apply(target, 'R', seed + 101 if base != "svd" else seed + 202, k)
    if target is not A:
        from ..models.aux import copy
        copy(target, A)
    return sv


def _fill(A, k, seed, scale):
    s = A.storage
    bc = s.bc
    if bc is None:
        # per-tile storage: generate tile by tile with its global offsets
        for (i, j, slot) in list(s.tiles.keys()):
            t = s.tiles[(i, j, slot)]
            ops.matgen(k, seed, t, s.m, s.n, max(t.shape[0], 1), 1, 0, max(t.shape[1], 1), 1, 0,
                       s.row_offsets[i], s.col_offsets[j], scale)
            s.table.modified(i, j, slot, True)
        return A
    if not s.local:
        A.insertLocalTiles(device=s.device if s.device.type == "cuda" else -1)
    slot = s.origin_slot
    if bc.pr < 0:
        return A
    lb = A.local_block(slot)
    # generate the view's local block with its absolute global coordinates;
    # indices are offsets into the full matrix so the result matches any view
    ops.matgen(k, seed, lb.data, s.m, s.n, bc.mb, bc.p, bc.pr, bc.nb, bc.q, bc.pc, 0, 0, scale) \
        if (lb.row_off == 0 and lb.col_off == 0) else \
        _gen_offset(k, seed, lb, s, bc, scale)
    s.mark_local_modified(slot)
    return A


def _gen_offset(k, seed, lb, s, bc, scale):
    # local block starting at local (row_off, col_off): the kernel's
    # local->global map assumes local index 0 at tile start, so generate the
    # enclosing tile-aligned block and copy the needed part.
    r_al = (lb.row_off // bc.mb) * bc.mb
    c_al = (lb.col_off // bc.nb) * bc.nb
    full = s.local[s.origin_slot]
    big = full[r_al:lb.row_off + lb.mloc, c_al:lb.col_off + lb.nloc]
    tmp = ops.colmajor_empty(big.shape[0], big.shape[1], big.dtype, big.device)
    # global of local r_al: l2g(r_al) = ((r_al/mb)*p + pr)*mb -> pass as row0 with a 1-tile-per-proc map
    from ..core.storage import l2g
    ops.matgen(k, seed, tmp, s.m, s.n, bc.mb, bc.p, bc.pr, bc.nb, bc.q, bc.pc,
               l2g(r_al, bc.mb, bc.pr, bc.p) - bc.pr * bc.mb, l2g(c_al, bc.nb, bc.pc, bc.q) - bc.pc * bc.nb,
               scale)
    lb.data.copy_(tmp[lb.row_off - r_al:, lb.col_off - c_al:])
