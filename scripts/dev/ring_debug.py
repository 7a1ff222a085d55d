"""Dev check: kinetic energy of each iteration's momentum recovered from E_chain (wu=0, no
integration: L in [0,1) -> no leapfrog, q unchanged) vs the host-regenerated normals."""
import sys, os
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "understanding-hmc_amd"), os.path.join(ROOT, "tests")]
from hmc_amd.engine import RandomEngine
from hmc_amd.target import MVNTarget
from test_gpu_philox_parity import gpu_normals
N, D, Niter, seed = 4, 100, 12, 77
eng = RandomEngine(MVNTarget(np.zeros(D), np.eye(D)), N, Niter, 0, 1, 0, 1, 0.1, rng="philox", seed=seed,
                   fp_mode="exact", store_chain=True)
q = np.random.RandomState(1).standard_normal((N, D))
eng.init(q)
eng.run(1, Niter + 1)
torch.cuda.synchronize()
E = eng.E_chain.cpu().numpy()
logc = D * np.log(2 * np.pi)
for it in range(1, Niter + 1):
    p = gpu_normals(seed, 0, N, it, 50)[:, :D]
    # E_chain[:, it-1] holds E0 of iteration it (wu = 0: row it-1 ... row index = it - wu = it)
    K_dev = 2 * E[:, it] - logc - (eng.q_chain.cpu().numpy()[:, it - 1] ** 2).sum(1)
    print(it, np.abs(K_dev - (p ** 2).sum(1)).max())
