"""The tester CLI (reference test/test + run_tests.py) runs and checks."""
import pytest

from slate_amd import tester


@pytest.mark.parametrize("routine", sorted(tester.ROUTINES))
def test_tester_routine(routine):
    assert tester.main([routine, "--type", "d,z", "--dim", "40x30x20", "--nb", "16", "--target", "h"]) == 0


def test_parse_dims():
    assert tester.parse_dims(["100:300:100"]) == [(100, 100, 100), (200, 200, 200), (300, 300, 300)]
    assert tester.parse_dims(["10x20x30"]) == [(10, 20, 30)]
