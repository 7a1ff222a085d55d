"""Dev A/B timing of the dense (c3) kernel, not a bench line: HMC_LIB_PATH selects the build.
usage: python scripts/dev/ab_dense.py [N] [K] [D] [rho]"""
import os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "understanding-hmc_amd")]
from hmc_amd.engine import RandomEngine
from hmc_amd.target import MVNTarget
from hmc_amd import _lib as H
a = sys.argv[1:] + ["262144", "10", "100", "0.95"][len(sys.argv) - 1:]
N, K, D, rho = int(a[0]), int(a[1]), int(a[2]), float(a[3])
cov = (1 - rho) * np.eye(D) + rho
eng = RandomEngine(MVNTarget(np.zeros(D), cov), N, K + 3, 0, 1, 5, 20, 0.1, rng="philox", seed=0, fp_mode="fast",
                   store_chain=False)
eng.init(torch.as_tensor(np.random.RandomState(0).standard_normal((N, D)) @ np.linalg.cholesky(cov).T).cuda())
eng.run(1, 3)
torch.cuda.synchronize()
c0 = eng.read_counters()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); eng.run(3, 3 + K); e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / K
lf = (eng.read_counters() - c0)[H.CNT_LEAPFROG]
print(f"{os.environ.get('HMC_LIB_PATH', 'libhmc.so')}: dense N={N} D={D} rho={rho}: {ms:.3f} ms/iteration, "
      f"{lf / K / (ms / 1e3):.4e} lf/s")
