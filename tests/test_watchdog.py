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


def test_driver_steps_beat():
    n0 = wd.last_beat()[2]
    A = sl.HermitianMatrix(sl.Uplo.Lower, 64, nb=16, device=torch.device("cpu"))
    A.insertLocalTiles()
    sl.generate_matrix(A, "poev", seed=1)
    assert sl.potrf(A, {sl.Option.Target: sl.Target.HostTask}) == 0
    tag, age, n = wd.last_beat()
    assert n > n0 and tag.startswith("potrf")
    assert not wd.inside()          # every region left
