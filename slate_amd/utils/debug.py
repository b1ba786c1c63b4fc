"""Debug helpers (`src/auxiliary/Debug.hh:15-77`, `Debug.cc`): tile /
MOSI-state dumps, memory-pool leak checks, matrix diffs.  Off unless
`Debug.on()` (or SLATE_AMD_DEBUG=1)."""
from __future__ import annotations

import os

import torch

from ..core.storage import DEV, HOST


class Debug:
    _on = os.environ.get("SLATE_AMD_DEBUG", "0") not in ("0", "")

    @classmethod
    def on(cls):
        cls._on = True

    @classmethod
    def off(cls):
        cls._on = False

    @classmethod
    def enabled(cls):
        return cls._on

    @staticmethod
    def tile_states(A) -> str:
        """One character per local tile and slot: M(odified) S(hared)
        O(n hold) I(nvalid) . (absent) -- SLATE printTilesMOSI."""
        from .. import _native
        s = A.storage
        H = _native._host
        MOD, SH, INV, HOLD = H.MOSI_Modified, H.MOSI_Shared, H.MOSI_Invalid, H.MOSI_OnHold

        def code(st):
            c = "M" if st & MOD else ("S" if st & SH else ("I" if st & INV else "?"))
            return c.lower() if st & HOLD else c
        lines = []
        for slot, name in ((HOST, "host"), (DEV, "dev")):
            rows = []
            for i in range(A.mt()):
                row = []
                for j in range(A.nt()):
                    gi, gj = A._global_ij(i, j)
                    if not s.tileIsLocal(gi, gj):
                        row.append(" ")
                    elif s.tileExists(gi, gj, slot):
                        st = s.table.state(gi, gj, slot)
                        row.append(code(int(st)))
                    else:
                        row.append(".")
                rows.append("".join(row))
            lines.append(f"{name}:\n" + "\n".join(rows))
        return "\n".join(lines)

    @staticmethod
    def check_mosi(storage, values=True) -> list:
        """MOSI coherency checker (SURVEY §5.2 race/consistency detection;
        SLATE checks the same invariants with asserts in MatrixStorage.hh):
        for every local tile (a) at most one copy is Modified, (b) a
        Modified copy has only Invalid siblings, (c) no copy is left OnHold,
        and with ``values`` (d) copies that are both valid hold equal data.
        Returns the violations as strings (empty: coherent)."""
        from .. import _native
        H = _native._host
        MOD, SH, INV, HOLD = H.MOSI_Modified, H.MOSI_Shared, H.MOSI_Invalid, H.MOSI_OnHold
        s = storage
        bad = []
        per = {}
        for (i, j, slot) in s.table.instances():
            if s.tileIsLocal(i, j):
                per.setdefault((i, j), {})[slot] = int(s.table.state(i, j, slot))
        for (i, j), st in per.items():
            mods = [x for x, v in st.items() if v & MOD]
            if len(mods) > 1:
                bad.append(f"tile ({i},{j}): Modified in slots {mods}")
            if mods and any(not (v & INV) for x, v in st.items() if x != mods[0]):
                bad.append(f"tile ({i},{j}): Modified in slot {mods[0]} but a sibling is still valid {st}")
            if any(v & HOLD for v in st.values()):
                bad.append(f"tile ({i},{j}): left OnHold {st}")
            if values and len(st) > 1:
                valid = [x for x, v in st.items() if not (v & INV)]
                if len(valid) > 1:
                    a = s.tile_data(i, j, valid[0])
                    b = s.tile_data(i, j, valid[1])
                    if a is not None and b is not None and not torch.equal(a.cpu(), b.cpu()):
                        bad.append(f"tile ({i},{j}): valid copies in slots {valid} differ")
        return bad

    @staticmethod
    def assert_mosi(storage, where=""):
        bad = Debug.check_mosi(storage)
        if bad:
            from ..core.exceptions import SlateError
            raise SlateError(f"MOSI check failed{(' after ' + where) if where else ''}: " + "; ".join(bad[:8]))

    @staticmethod
    def check_pool_leaks(*matrices) -> dict:
        """Workspace blocks still handed out by the matrices' slab pools
        (checkDeviceMemoryLeaks analog, src/core/Memory.cc:111): after a
        driver released its workspace every count should be 0."""
        out = {}
        for A in matrices:
            st = A.storage
            for slot in list(st.pools):
                stats = st.pool_stats(slot)
                out[(id(st), slot)] = int(stats.get("in_use", 0))
        return out

    @staticmethod
    def diff(A, B, tol=0.0):
        """Positions (i, j) where the gathered A and B differ by > tol."""
        from ..models.aux import allgather_dense
        X, Y = allgather_dense(A), allgather_dense(B)
        d = (X - Y).abs()
        idx = (d > tol).nonzero().tolist()
        return idx, float(d.max()) if d.numel() else 0.0

    @staticmethod
    def diff_lapack(A: torch.Tensor, B: torch.Tensor, mb=None, nb=None, tol=0.0) -> str:
        """Tile map of differences between two dense matrices (diffLapackMatrices)."""
        m, n = A.shape
        mb = mb or m
        nb = nb or n
        lines = []
        for i0 in range(0, m, mb):
            row = []
            for j0 in range(0, n, nb):
                dd = (A[i0:i0 + mb, j0:j0 + nb] - B[i0:i0 + mb, j0:j0 + nb]).abs().max().item()
                row.append("X" if dd > tol else ".")
            lines.append("".join(row))
        return "\n".join(lines)
