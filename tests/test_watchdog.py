"""Progress/communication watchdog: heartbeats from Comm
collectives and driver steps; a stalled rank is reported with its last step."""
import time

import torch

import slate_amd as sl
from slate_amd.utils import watchdog as wd


def test_watchdog_fires_on_stall():
    seen = []
    w = sl.Watchdog(0.3, abort=False, callback=seen.append, poll=0.05).start()
    wd.enter("potrf")
    try:
        wd.beat("potrf step 3")
        time.sleep(1.0)
    finally:
        wd.leave("potrf")
        w.stop()
    assert seen and seen[0]["tag"] == "potrf step 3" and seen[0]["age_s"] > 0.3


def test_watchdog_quiet_outside_library():
    """Application time outside any slate_amd region never fires it
    (an armed watchdog killed healthy ranks between calls)."""
    seen = []
    w = sl.Watchdog(0.2, abort=False, callback=seen.append, poll=0.05).start()
    assert not wd.inside()
    time.sleep(0.8)
    w.stop()
    assert not seen


def test_watchdog_quiet_while_beating():
    seen = []
    with sl.Watchdog(0.5, abort=False, callback=seen.append, poll=0.05):
        for _ in range(12):
            wd.beat("tick")
            time.sleep(0.05)
    assert not seen


def test_watchdog_fires_in_comm_call_outside_driver():
    """a collective issued outside any driver (a timing barrier,
    finalize, user-level comm) is a library region: a peer lost there fires
    the watchdog.  The hang is simulated by a Comm method that sleeps."""
    from slate_amd.parallel.comm import Comm

    class Stuck(Comm):
        def __init__(self):
            pass

        @wd.watched("comm.barrier")
        def barrier(self):
            time.sleep(1.0)

    seen = []
    w = sl.Watchdog(0.3, abort=False, callback=seen.append, poll=0.05).start()
    try:
        assert not wd.inside()
        Stuck().barrier()
    finally:
        w.stop()
    assert seen and seen[0]["tag"] == "comm.barrier"
    assert not wd.inside()


def test_comm_methods_are_watched_regions():
    from slate_amd.parallel.comm import Comm
    for name in ("barrier", "bcast", "allreduce", "allgather", "reduce", "send", "recv", "exchange"):
        assert getattr(Comm, name).__wrapped__ is not None, name


def test_watchdog_depth_thread_safe():
    import threading

    def worker():
        for _ in range(2000):
            wd.enter("x")
            wd.leave("x")

    ts = [threading.Thread(target=worker) for _ in range(8)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not wd.inside()


def test_driver_steps_beat():
    n0 = wd.last_beat()[2]
    A = sl.HermitianMatrix(sl.Uplo.Lower, 64, nb=16, device=torch.device("cpu"))
    A.insertLocalTiles()
    sl.generate_matrix(A, "poev", seed=1)
    assert sl.potrf(A, {sl.Option.Target: sl.Target.HostTask}) == 0
    tag, age, n = wd.last_beat()
    assert n > n0 and tag.startswith("potrf")
    assert not wd.inside()          # every region left
