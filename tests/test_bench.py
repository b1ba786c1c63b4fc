"""bench.py contract on the CPU: one JSON line from rank 0 with the
driver's fields, single rank and 2 ranks (gloo, 127.0.0.1) -- the same code
path the driver runs per GPU count (RCCL there)."""
import json
import os
import subprocess
import sys

import pytest

from dist_util import _free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _run(nproc, routine, self_launch=False, expect_rc=0):
    args = ["bench.py", "--gpus", str(nproc), "--routine", routine, "--size", "512", "--nb", "64", "--steps", "1",
            "--warmup", "1"]
    if routine == "geqrf":
        args += ["--rows", "768"]
    if nproc > 1 and not self_launch:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", f"--master-port={_free_port()}"] + args
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    if expect_rc != 0:
        assert out.returncode != 0
        return out
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("nproc", [1, 2])
@pytest.mark.parametrize("routine", ["potrf", "getrf", "geqrf"])
def test_bench_json(nproc, routine):
    d = _run(nproc, routine)
    assert KEYS <= set(d)
    assert d["n_gpus"] == nproc and d["steps"] == 1 and d["warmup"] == 1
    assert d["value"] > 0 and d["higher_is_better"] is True
    assert d["config"]["n"] == 512
    if nproc == 1:
        assert d["residual"] is not None and d["residual"] < 1e-12


@pytest.mark.parametrize("nproc,grid", [(4, "2x2"), (8, "2x4")])
@pytest.mark.parametrize("routine", ["potrf", "getrf"])
def test_bench_json_many_ranks(nproc, grid, routine):
    """The driver's N = 4 / 8 launches: the default grids (BASELINE: 2x4 at
    8 GPUs), one JSON line, info 0 on every rank."""
    d = _run(nproc, routine)
    assert KEYS <= set(d)
    assert d["n_gpus"] == nproc and d["config"]["grid"] == grid
    assert d["info_ok"] is True and d["value"] > 0


@pytest.mark.parametrize("nproc,grid", [(4, "2x2"), (8, "2x4")])
def test_bench_self_launch(nproc, grid):
    """``python bench.py --gpus N`` without a launcher
    starts N ranks itself (one process per GPU) and rank 0's JSON line
    reports the N-rank run."""
    d = _run(nproc, "potrf", self_launch=True)
    assert d["n_gpus"] == nproc and d["config"]["grid"] == grid
    assert d["info_ok"] is True and d["residual_ok"] is True


def test_bench_world_mismatch_is_an_error():
    """--gpus 2 under a 1-rank environment is refused, not silently measured
    on one GPU."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--size", "256", "--nb", "64", "--steps", "1",
                          "--warmup", "0"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


def test_potrf_plan_prologue_fast():
    """the 2 x 4 dpotrf (n = 32768, nb = 512) column-gather
    plans cost ~40 ms of host Python per call.  Now built with numpy range
    arithmetic and cached per geometry: a repeated call (every bench step
    after the first) is a dictionary lookup, < 1 ms."""
    import time
    from slate_amd.models._panels import plan_col_gathers_steps
    n, nb, p, q = 32768, 512, 2, 4
    nt = n // nb
    tm = lambda j: nb                  # noqa: E731
    for pc in range(q):
        plan_col_gathers_steps(tm, 0, nt, nb, p, q, pc, "cpu", split=1)     # first call builds
    t0 = time.perf_counter()
    for pc in range(q):
        plans = plan_col_gathers_steps(tm, 0, nt, nb, p, q, pc, "cpu", split=1)
    dt = (time.perf_counter() - t0) / q
    assert len(plans) == nt
    assert dt < 1e-3, f"{dt * 1e3:.2f} ms per call"
