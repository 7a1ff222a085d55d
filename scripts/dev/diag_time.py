"""Dev timing of convergence_stats on a bench-shaped window (not a bench line):
python scripts/dev/diag_time.py [N] [R] [D] [reps]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "understanding-hmc_amd")]
from hmc_amd import diagnostics as G  # noqa: E402

a = sys.argv[1:] + ["1048576", "100", "100", "3"][len(sys.argv) - 1:]
N, R, D, reps = (int(x) for x in a[:4])
g = torch.Generator(device="cuda").manual_seed(1)
x = torch.randn((N, R, D), dtype=torch.float64, device="cuda", generator=g)
for k in range(1, R):                               # AR(1)-ish rows: lags matter
    x[:, k].mul_(0.6).add_(x[:, k - 1], alpha=0.4)
torch.cuda.synchronize()
for r in range(reps):
    t0 = time.perf_counter()
    Rh, ne = G.convergence_stats(x, warm_up_num=0, thin_rate=1)
    torch.cuda.synchronize()
    print(f"rep {r}: {time.perf_counter() - t0:.4f} s  info={G.LAST_INFO}  rhat_med={np.median(Rh):.5f} "
          f"neff_med={np.median(ne):.4e}", flush=True)
