"""Matrix printing (`include/slate/print.hh:23-120`, `src/print.cc`):
`print(label, A, opts)` with Option.PrintVerbose (0 none, 1 metadata,
2 edge items, 3 + tile boundaries, 4 everything), PrintEdgeItems,
PrintWidth, PrintPrecision.  The matrix is gathered to rank 0 (the only
rank that prints), like SLATE's rank-0 gathers."""
from __future__ import annotations

import io
import sys

import torch

from ..core.enums import Option
from ..core.options import get_option


def _fmt(v, width, prec):
    if isinstance(v, complex):
        return f"{v.real:{width}.{prec}f} + {v.imag:{width}.{prec}f}i"
    return f"{v:{width}.{prec}f}"


def format_matrix(label, A, opts=None) -> str:
    from ..models.aux import allgather_dense
    verbose = int(get_option(opts, Option.PrintVerbose, 4))
    edge = int(get_option(opts, Option.PrintEdgeItems, 16))
    width = int(get_option(opts, Option.PrintWidth, 10))
    prec = int(get_option(opts, Option.PrintPrecision, 4))
    out = io.StringIO()
    m, n = A.m(), A.n()
    s = A.storage
    grid = f"{s.bc.p}x{s.bc.q}" if s.bc is not None else "general"
    if verbose == 0:
        return ""
    out.write(f"% {label}: {type(A).__name__} {m}-by-{n}, {A.mt()}-by-{A.nt()} tiles, "
              f"tile size {A.tileMb(0) if A.mt() else 0}-by-{A.tileNb(0) if A.nt() else 0}, grid {grid}, "
              f"op {A.op().name}, uplo {A.uplo().name}, dtype {s.dtype}\n")
    if verbose == 1:
        return out.getvalue()
    D = allgather_dense(A).cpu()
    rows = list(range(m))
    cols = list(range(n))
    if verbose == 2:
        if m > 2 * edge:
            rows = list(range(edge)) + [-1] + list(range(m - edge, m))
        if n > 2 * edge:
            cols = list(range(edge)) + [-1] + list(range(n - edge, n))
    nb = A.tileNb(0) if A.nt() else n
    mb = A.tileMb(0) if A.mt() else m
    out.write(f"{label} = [\n")
    for i in rows:
        if i == -1:
            out.write("  ...\n")
            continue
        if verbose >= 3 and i and i % mb == 0:
            out.write("\n")
        parts = []
        for j in cols:
            if j == -1:
                parts.append("...")
                continue
            if verbose >= 3 and j and j % nb == 0:
                parts.append("  ")
            v = D[i, j].item()
            parts.append(_fmt(v, width, prec))
        out.write("  " + " ".join(parts) + "\n")
    out.write("];\n")
    return out.getvalue()


def print_matrix(label, A, opts=None, file=None):
    """Print A (rank 0 only; all ranks must call: the gather is collective)."""
    txt = format_matrix(label, A, opts)
    if A.storage.comm.rank in (0, -1) or A.storage.comm.size == 1:
        (file or sys.stdout).write(txt)
        (file or sys.stdout).flush()
    return txt


def print_vector(label, x, opts=None, file=None):
    prec = int(get_option(opts, Option.PrintPrecision, 4))
    v = torch.as_tensor(x).reshape(-1).cpu().tolist()
    txt = f"{label} = [ " + " ".join(_fmt(e, 1, prec) for e in v) + " ];\n"
    (file or sys.stdout).write(txt)
    return txt
