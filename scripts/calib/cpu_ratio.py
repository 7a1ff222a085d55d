"""Restatement-to-reference CPU speed ratio (BASELINE.md §3 "Calibration"): BUILD CONTAINER ONLY.

Times the reference's own HMC_sampler (loaded in memory from /root/reference by
tests/golden/make_golden.py's loader; nothing of its source is written anywhere) and the
oracle restatement (oracle/hmc_oracle.py, the engine bench.py's cpu_baseline leg runs on the
GPU box) on the same single-chain workload bench.py's worker uses: 1 chain, 20-iteration
rounds, L ~ U{5..19}, dt 0.1, one BLAS thread, leapfrogs counted exactly.
Usage: OMP_NUM_THREADS=1 OPENBLAS_NUM_THREADS=1 python scripts/calib/cpu_ratio.py [seconds]"""
import contextlib
import io
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import make_golden as MG          # noqa: E402  (loads the reference in memory)
from oracle import hmc_oracle as O  # noqa: E402

BUDGET = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0


def time_reference(D, rho, sampler):
    q0, cov0, inv_cov0, V, dVdq = MG.mvn_target(D, rho)
    np.random.seed(1000)
    q = MG.ref_utils.start_pts(q0, 2 * np.eye(D), 1)
    lf, t0 = 0, time.time()
    while time.time() - t0 < BUDGET:
        if sampler == "nuts":
            h = MG.ref_samplers.HMC_sampler(D, V, dVdq, Niter=2, Nchain=1, sampler_type="NUTS", dt=0.1, d_max=12)
        else:
            h = MG.ref_samplers.HMC_sampler(D, V, dVdq, Niter=20, Nchain=1, sampler_type="Random", L_low=5,
                                            L_high=20, dt=0.1)
        n = [0]
        f = h.leap_frog

        def counted(p, qq):
            n[0] += 1
            return f(p, qq)
        h.leap_frog = counted
        with contextlib.redirect_stdout(io.StringIO()):
            h.gen_sample(q, verbose=False)
        lf += n[0]
        q = h.q_chain[:, -1, :]
    return lf / (time.time() - t0)


def time_oracle(D, rho, sampler):
    np.random.seed(1000)
    cov = np.eye(D) if rho == 0 else O.mvn_cov(D, rho)
    core = O.HMCCore(O.MVNTarget(np.zeros(D), cov), 0.1)
    q = O.start_pts(np.zeros(D), 2 * np.eye(D), 1)
    lf, t0 = 0, time.time()
    while time.time() - t0 < BUDGET:
        if sampler == "nuts":
            out = O.gen_sample_nuts(core, q, 1, 2, 0, 1, 12, O.LiveDraws(D, np.eye(D)), on_dmax="break")
        else:
            out = O.gen_sample_random(core, q, 1, 20, 0, 1, 5, 20, O.LiveDraws(D, np.eye(D)))
        lf += out["n_leapfrog"]
        q = out["q_chain"][:, -1, :]
    return lf / (time.time() - t0)


rows = []
for D, rho, sampler in ((100, 0.0, "random"), (100, 0.95, "random"), (100, 0.95, "nuts")):
    r, o = time_reference(D, rho, sampler), time_oracle(D, rho, sampler)
    rows.append(dict(D=D, rho=rho, sampler=sampler, reference_lf_s=r, oracle_lf_s=o, oracle_over_reference=o / r))
    print(json.dumps(rows[-1]), flush=True)
cpu = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")), "?")
print(json.dumps(dict(cpu_model=cpu, numpy=np.__version__, budget_s=BUDGET, threads=1)))
