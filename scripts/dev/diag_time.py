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

# the one-pass kernel alone, per lag width (HIP events), with board power / clock while it runs
if os.environ.get("DIAG_KERNEL"):
    from bench import Telemetry  # noqa: E402
    sp = G._Split(x, 1, 0)
    for tm in [int(t) for t in os.environ["DIAG_KERNEL"].split(",")]:
        G.convergence_sums(sp, tm)
        torch.cuda.synchronize()
        tel = Telemetry(0, 0.005).start()
        ts = []
        for r in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            G.convergence_sums(sp, tm)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(f"tmax {tm}: ms {[round(t, 2) for t in ts]}  telemetry {tel.stop()}", flush=True)
