"""Dev A/B timing of the diagonal Random kernel (not a bench line): HMC_LIB_PATH selects the build.
usage: python scripts/dev/ab_wave.py [N] [S] [K] [D] [window_rows] [reps]
(reps > 1 re-runs the same K launches, for power/clock sampling over a longer run)"""
import os, sys, time
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "understanding-hmc_amd")]
from hmc_amd.engine import RandomEngine
from hmc_amd.target import MVNTarget
from hmc_amd import _lib as H
N, S, K, D, R, REPS = [int(x) for x in (sys.argv[1:] + ["1048576", "40", "10", "100", "100", "1"][len(sys.argv) - 1:])]
W = 2
eng = RandomEngine(MVNTarget(np.zeros(D), np.eye(D)), N, (W + K) * S, W * S + 1, 1, 5, 20, 0.1, rng="philox", seed=0,
                   fp_mode="fast", store_chain=False)
if R > 0:
    win = torch.zeros((N, R, D), dtype=torch.float64, device="cuda")
    eng.set_chain_window(win, 0)
eng.init(torch.randn(N, D, dtype=torch.float64, device="cuda"))
it = 1
for _ in range(W):
    eng.run(it, it + S); it += S
torch.cuda.synchronize()
c0 = eng.read_counters()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K * REPS)]
it_start = it
for r in range(REPS):
    it = it_start
    for k in range(K):
        e = ev[r * K + k]
        e[0].record(); eng.run(it, it + S); e[1].record(); it += S
torch.cuda.synchronize()
ms = np.mean([a.elapsed_time(b) for a, b in ev])
lf = (eng.read_counters() - c0)[H.CNT_LEAPFROG] / REPS
print(f"{os.environ.get('HMC_LIB_PATH', 'libhmc.so')}: N={N} S={S} D={D} R={R}: {ms:.3f} ms/launch, "
      f"{lf / K / (ms / 1e3):.4e} lf/s")
