"""The reference's case studies (case1-script.py ... case5-script.py, case3-script-2.py) as
Python-3 drivers of the MI355X engine.

Each reference script runs one target family at D = 2, 10, 100 (variants a, b, c):
  case 1: unit MVN                     case 2: unit MVN, far starts (chain 0 at (1000, -750, 0...))
  case 3: rho = 0.95 (3-2: D=100, L in [50, 200))
  case 4: rho = 0.99                   case 5: rho = 0.999
with Niter 2000, 10 chains, warm-up 1000, thin 1, dt 0.1, L ~ U{5..19}, 100 saved chain-0
trajectories, starts ~ N(q0, 2I) (x100 for case 2).  The driver builds the same V/dVdq
closures and calls the same HMC_sampler surface; the sampler probes the closures into an MVN
descriptor and runs the fused HIP kernels.  Like every reference script, a run ends with
plot_samples (savefig, the 3x3 summary PNG) and make_movie (the chain-0 PNG deck) on the
GPU-filled sampler (case1-script.py:66-67), written under --out-dir as the reference's
./caseN/caseNx prefixes; --no-plots skips them, --movie-frames caps the deck.

    python drivers/cases.py 1a [--seed 0] [--chains N --rng philox] [--sampler NUTS] [--no-plots]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "understanding-hmc_amd"))

COMMON = dict(Niter=2000, Nchain=10, warm_up=1000, thin=1, n_save=100, dt=0.1, L_low=5, L_high=20,
              start_scale=2.0, far_chain0=False)
FAMILY = {"1": dict(rho=0.0), "2": dict(rho=0.0, start_scale=100.0, far_chain0=True), "3": dict(rho=0.95),
          "4": dict(rho=0.99), "5": dict(rho=0.999)}
CASES = {f"{k}{v}": dict(COMMON, D=d, **FAMILY[k]) for k in FAMILY for v, d in (("a", 2), ("b", 10), ("c", 100))}
CASES["3-2"] = dict(COMMON, D=100, rho=0.95, L_low=50, L_high=200)     # case3-script-2.py


def target(D, rho):
    """q0 = 0, cov0 = (1 - rho) I + rho 11^T and the closures V = -lnL, dVdq = inv(cov0) (q - q0)."""
    from hmc_amd.utils import normal_lnL
    q0 = np.zeros(D)
    cov0 = np.diag(np.ones(D)) * (1 - rho) + rho
    inv_cov0 = np.linalg.inv(cov0)

    def V(q):
        return -normal_lnL(q, q0, cov0)

    def dVdq(q):
        return np.dot(inv_cov0, (q - q0))
    return q0, cov0, V, dVdq


def title_prefix(name, out_dir="."):
    """The reference's title_str: ./case1/case1a ... (case3-script-2.py: ./case3/case3d)."""
    fam = name.split("-")[0][0]
    tag = "3d" if name == "3-2" else name
    return os.path.join(out_dir, "case%s" % fam, "case%s" % tag)


def run_case(name, seed=None, chains=None, rng="replay", sampler="Random", d_max=10, verbose=True,
             fp_mode="exact", plots=False, out_dir=".", movie_frames=None, movie_dpi=200):
    """Run one case; returns the HMC_sampler (reference attributes filled).  plots=True ends the
    run as the reference scripts do (case1-script.py:66-67): plot_samples(savefig) and make_movie
    into title_prefix(name, out_dir); h.plot_summary / h.movie_files hold what they drew."""
    from hmc_amd.samplers import HMC_sampler
    from hmc_amd.utils import start_pts
    c = dict(CASES[name])
    if chains:
        c["Nchain"] = int(chains)
    D, Nchain = c["D"], c["Nchain"]
    if seed is not None:
        np.random.seed(seed)
    q0, cov0, V, dVdq = target(D, c["rho"])
    if verbose:
        print("#---- Case %s (D=%d, rho=%.3f, %d chains) ----#" % (name, D, c["rho"], Nchain))
        print("Min/Max of marginal variances: %.3f, %.3f" % (np.min(np.diag(cov0)), np.max(np.diag(cov0))))
    q_start = start_pts(q0, np.diag(np.ones(D)) * c["start_scale"], Nchain)
    if c["far_chain0"]:
        q_start[0, :] = 0
        q_start[0, 0] = 1000
        q_start[0, 1] = -750
    kw = dict(Niter=c["Niter"], Nchain=Nchain, dt=c["dt"], thin_rate=c["thin"], warm_up_num=c["warm_up"], rng=rng,
              seed=0 if seed is None else seed, fp_mode=fp_mode)
    if sampler == "NUTS":
        h = HMC_sampler(D, V, dVdq, sampler_type="NUTS", d_max=d_max, **kw)
    else:
        h = HMC_sampler(D, V, dVdq, sampler_type="Random", L_low=c["L_low"], L_high=c["L_high"], **kw)
    t0 = time.time()
    h.gen_sample(q_start, N_save_chain0=c["n_save"] if sampler != "NUTS" else 0, verbose=verbose)
    wall = time.time() - t0
    h.compute_convergence_stats()
    if verbose:
        total = (h.L_chain - 1) * h.Nchain
        print(sampler)
        print("Total number of samples: %d" % total)
        print("Effective number per param: ", h.n_eff_q)
        print("Ratio", h.n_eff_q / total)
        print("R-hat: ", h.R_q)
        print("leapfrog steps: %d in %.3f s (%.3e /s incl. host streams and copies)"
              % (h.n_leapfrog, wall, h.n_leapfrog / wall))
    h.plot_summary, h.movie_files = None, None
    if plots:
        title = title_prefix(name, out_dir)
        os.makedirs(os.path.dirname(title), exist_ok=True)
        h.plot_summary = h.plot_samples(title_prefix=title, savefig=True, show=False, plot_normal=True, q0=q0,
                                        cov0=cov0)
        if sampler == "Random":                          # the reference's movie is Random-only (:850)
            lim = 1100 if c["far_chain0"] else 4         # case2-script.py:69 / case1-script.py:67
            h.movie_files = h.make_movie(title_prefix=title, q0=q0, cov0=cov0, plot_cov=True, qmin=-lim, qmax=lim,
                                         max_frames=movie_frames, dpi=movie_dpi)
    if verbose:
        print()
    return h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case", nargs="+", choices=sorted(CASES))
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--chains", type=int, default=None)
    ap.add_argument("--rng", default="replay", choices=["replay", "philox"])
    ap.add_argument("--sampler", default="Random", choices=["Random", "NUTS"])
    ap.add_argument("--d-max", type=int, default=10)
    ap.add_argument("--fp-mode", default="exact", choices=["exact", "fast"])
    ap.add_argument("--no-plots", action="store_true", help="skip plot_samples / make_movie")
    ap.add_argument("--out-dir", default=".", help="where the ./caseN/caseNx figure prefixes go")
    ap.add_argument("--movie-frames", type=int, default=None, help="cap on make_movie slides (default: all)")
    a = ap.parse_args()
    for name in a.case:
        run_case(name, seed=a.seed, chains=a.chains, rng=a.rng, sampler=a.sampler, d_max=a.d_max, fp_mode=a.fp_mode,
                 plots=not a.no_plots, out_dir=a.out_dir, movie_frames=a.movie_frames)


if __name__ == "__main__":
    main()
