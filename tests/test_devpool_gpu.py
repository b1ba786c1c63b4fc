"""Native stream-ordered device slab pool (csrc/hip/devpool.hip) -- the
Memory-class analog (reference src/core/Memory.cc:17-220)."""
import pytest
import torch

from slate_amd import _native

pytestmark = pytest.mark.gpu


def test_devpool_reuse_and_cap():
    hip = _native.hip()
    pool = hip.DevicePool(0, 4000, 4, 0)
    assert pool.block_bytes() == 4096                    # 256-byte aligned blocks
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    c, i, off, grew = pool.alloc(s1.cuda_stream)
    assert grew and c == 0 and off == i * 4096
    raw = torch.utils.dlpack.from_dlpack(pool.chunk_view(0))
    assert raw.is_cuda and raw.numel() == 4 * 4096
    blk = raw[off:off + 4096].view(torch.float64)
    with torch.cuda.stream(s1):
        blk.fill_(3.0)
    pool.free(c, i, s1.cuda_stream)
    # same stream: handed out again at once (stream order)
    c2, i2, off2, grew2 = pool.alloc(s1.cuda_stream)
    assert not grew2 and (c2, i2) == (c, i)
    st = pool.stats()
    assert st["in_use"] == 1 and st["reuse_same_stream"] >= 1
    torch.cuda.synchronize()
    assert float(raw[off2:off2 + 4096].view(torch.float64).sum()) == 3.0 * 512
    pool.free(c2, i2, s1.cuda_stream)
    del raw, blk
    torch.cuda.synchronize()
    assert pool.trim() == 1 and pool.stats()["chunks"] == 0


def test_devpool_cap_orders_on_device():
    hip = _native.hip()
    pool = hip.DevicePool(0, 4096, 2, 8192)             # cap: one chunk of two blocks
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = pool.alloc(s1.cuda_stream)
    b = pool.alloc(s1.cuda_stream)
    with pytest.raises(RuntimeError, match="HBM cap"):
        pool.alloc(s2.cuda_stream)
    # a long kernel on s1, then free there; s2 gets the block ordered after it
    x = torch.randn(2048, 2048, device="cuda", dtype=torch.float64)
    with torch.cuda.stream(s1):
        for _ in range(4):
            x = x @ x / 2048.0
    pool.free(a[0], a[1], s1.cuda_stream)
    c = pool.alloc(s2.cuda_stream)
    assert (c[0], c[1]) == (a[0], a[1])
    st = pool.stats()
    assert st["device_waits"] + st["reuse_completed"] == 1
    pool.free(c[0], c[1], s2.cuda_stream)
    pool.free(b[0], b[1], s1.cuda_stream)
    torch.cuda.synchronize()
    assert pool.stats()["in_use"] == 0


def test_storage_workspace_tiles_from_devpool():
    import slate_amd as sl
    from slate_amd.core.enums import TileKind
    A = sl.Matrix(1024, 1024, nb=256, device=torch.device("cuda", 0))
    st = A.storage
    DEV = 1
    st.tileInsert(0, 0, DEV, kind=TileKind.Workspace)
    st.tileInsert(1, 0, DEV, kind=TileKind.Workspace)
    t = st.tiles[(0, 0, DEV)]
    assert t.is_cuda and t.shape == (256, 256) and t.stride(0) == 1
    t.fill_(1.0)
    stats = st.pool_stats(DEV)
    assert stats["in_use"] == 2 and "device_waits" in stats
    st.tileErase(0, 0, DEV)
    st.tileErase(1, 0, DEV)
    assert st.pool_stats(DEV)["in_use"] == 0
    assert all(v == 0 for v in sl.Debug.check_pool_leaks(A).values()) if hasattr(sl, "Debug") else True
