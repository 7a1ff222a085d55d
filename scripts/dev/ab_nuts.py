"""Dev A/B timing of the NUTS kernel (not a bench line): HMC_LIB_PATH selects the build.
usage: python scripts/dev/ab_nuts.py [N] [S] [K] [D] [rho]"""
import os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "understanding-hmc_amd")]
from hmc_amd.engine import NutsEngine
from hmc_amd.target import MVNTarget
from hmc_amd import _lib as H
a = sys.argv[1:] + ["65536", "2", "4", "100", "0.95"][len(sys.argv) - 1:]
N, S, K, D, rho = int(a[0]), int(a[1]), int(a[2]), int(a[3]), float(a[4])
cov = (1 - rho) * np.eye(D) + rho
eng = NutsEngine(MVNTarget(np.zeros(D), cov), N, (K + 2) * S, 0, 1, 10, 0.1, rng="philox", seed=0, fp_mode="fast",
                 store_chain=False, on_dmax="break")
q0 = torch.as_tensor(np.random.RandomState(0).standard_normal((N, D)) @ np.linalg.cholesky(cov).T).cuda()
eng.init(q0)
it = 1
for _ in range(2):
    eng.run(it, it + S); it += S
torch.cuda.synchronize()
c0 = eng.read_counters()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
for k in range(K):
    ev[k][0].record(); eng.run(it, it + S); ev[k][1].record(); it += S
torch.cuda.synchronize()
ms = np.mean([x.elapsed_time(y) for x, y in ev])
c = eng.read_counters() - c0
lf = c[H.CNT_LEAPFROG]
print(f"{os.environ.get('HMC_LIB_PATH', 'libhmc.so')}: NUTS N={N} S={S} D={D}: {ms:.3f} ms/launch, "
      f"{lf / K / (ms / 1e3):.4e} lf/s, lane util {lf / (c[H.CNT_LEAPFROG_SQ] * 16):.3f}")
