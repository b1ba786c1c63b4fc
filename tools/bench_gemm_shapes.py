"""GEMM shape/transpose sweep: the QR trailing-update shapes (small m, huge k)."""
import sys
sys.path.insert(0, '.')
from tools.bench_gemm import run  # noqa: E402

for ta, tb in [('N', 'N'), ('T', 'N'), ('N', 'T'), ('T', 'T')]:
    run('d', ta, tb, 512, 16384, 16384, reps=3)
for ta, tb in [('N', 'N'), ('T', 'N')]:
    run('d', ta, tb, 8192, 8192, 8192, reps=3)
    run('d', ta, tb, 16384, 512, 16384, reps=3)
    run('d', ta, tb, 16384, 16384, 512, reps=3)
