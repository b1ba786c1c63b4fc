"""Every example runs (reference examples/run_tests.py)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_examples_single_process():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "run_examples.py")], cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=900)
    assert r.returncode == 0, r.stdout
