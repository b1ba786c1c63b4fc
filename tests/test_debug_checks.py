"""Debug / race-detection aids: the MOSI coherency checker,
the serial-stream mode, and the host-code sanitizer build."""
import os
import subprocess
import sys

import pytest
import torch

import slate_amd as sl
from slate_amd.utils.debug import Debug
from slate_amd.core.exceptions import SlateError


def test_mosi_checker_clean_drivers(monkeypatch):
    monkeypatch.setattr(Debug, "_on", True)
    A = sl.HermitianMatrix(sl.Uplo.Lower, 64, nb=16)
    A.insertLocalTiles()
    sl.generate_matrix(A, "poev", 1)
    assert sl.potrf(A) == 0                       # the checker runs inside (mark_local_modified)
    B = sl.Matrix(64, 64, nb=16)
    B.insertLocalTiles()
    sl.generate_matrix(B, "rands", 2)
    piv = sl.Pivots()
    assert sl.getrf(B, piv) == 0
    assert Debug.check_mosi(A.storage) == [] and Debug.check_mosi(B.storage) == []


def test_mosi_checker_detects_incoherence():
    from slate_amd import _native
    H = _native._host
    A = sl.Matrix(32, 32, nb=16)
    A.insertLocalTiles()
    sl.generate_matrix(A, "rands", 3)
    s = A.storage
    i, j = 0, 0
    slot = next(sl_ for (a, b, sl_) in s.table.instances() if (a, b) == (i, j))
    s.table.set_state(i, j, slot, H.MOSI_Modified | H.MOSI_OnHold)
    bad = Debug.check_mosi(s)
    assert any("OnHold" in b for b in bad)
    with pytest.raises(SlateError):
        Debug.assert_mosi(s, "test")


def test_host_asan_build_runs_host_kernels(tmp_path):
    """Host code under AddressSanitizer + UBSan: the native host module is
    rebuilt with -fsanitize=address,undefined (host only -- GPU sanitizers
    are not available on this pool) and a small host-kernel workload runs
    with libasan preloaded; any memory error aborts the child."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "asan", "run_host_asan.py"), str(tmp_path)],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=900)
    if r.returncode == 77:
        pytest.skip(r.stdout[-500:])
    assert r.returncode == 0, r.stdout[-4000:]
    assert "ASAN-OK" in r.stdout
