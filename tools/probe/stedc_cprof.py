"""Host-side profile (cProfile) of one stedc_rows call at n = 16384 on the
GPU: where the Python driver spends its time (syncs included)."""
import cProfile
import os
import pstats
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from slate_amd.models.stedc import stedc_rows  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
dev = torch.device("cuda")
rng = np.random.default_rng(0)
d, e = rng.standard_normal(n), rng.standard_normal(n - 1)
stedc_rows(d, e, None, dev)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
stedc_rows(d, e, None, dev)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(25)
st.sort_stats("tottime").print_stats(15)
