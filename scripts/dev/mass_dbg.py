"""Dev check (not a test): stationarity of Philox NUTS with full / diagonal cov_p across kernels."""
import sys, os, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "understanding-hmc_amd"), os.path.join(ROOT, "tests")]
from hmc_amd.engine import NutsEngine
from hmc_amd import _lib as H
from hmc_amd.target import MVNTarget
from oracle import hmc_oracle as O
import make_golden_shapes as S
for D in (100, 136, 330):
    cov = O.mvn_cov(D, 0.6)
    full = S.dense_cov_p(D)
    for name, cp in (("full", full), ("diag", np.diag(np.diag(full))), ("none", None)):
        N = 512
        qs = np.random.RandomState(4).standard_normal((N, D)) @ np.linalg.cholesky(cov).T
        e = NutsEngine(MVNTarget(np.zeros(D), cov), N, 3, 1, 1, 8, 0.2, cov_p=cp, rng="philox", seed=6,
                       on_dmax="break")
        e.init(qs); e.run(1, 4); torch.cuda.synchronize()
        last = e.q_chain.cpu().numpy()[:, -1, :]
        c = e.read_counters()
        print(D, name, "var", last.var(axis=0).mean(), "lf/it", c[H.CNT_LEAPFROG] / (N * 3), "dmax", c[H.CNT_DMAX],
              "unst", c[H.CNT_UNSTABLE], flush=True)
