"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Test infrastructure only — run in the build container, never on the GPU box.

The reference (jaekor91/understanding-HMC, read-only at /root/reference) is Python 2.
This script loads `/root/reference/utils.py` and `/root/reference/samplers.py`
*in memory*, applies the stdlib lib2to3 `print`/`xrange` fixers plus the one
semantic Python-2 fix (`utils.py:102` integer division `L_chain/2` -> `//`),
restores the removed NumPy aliases (`np.float`, `np.int`) and runs the
reference's own classes on small seeded cases.  Nothing of the reference source
is written anywhere; only data (inputs + outputs) is saved, as `.npz`/`.json`.

Random streams are captured by wrapping the three legacy global-RNG entry points
the reference calls (`np.random.multivariate_normal`, `randint`, `random`;
samplers.py:441, :461, :608, :748, :773, :829, utils.py:209) with pass-through
recorders, so the fixtures hold exactly the draws the reference consumed.

Usage:  python tests/golden/make_golden.py  (writes tests/golden/*.npz, *.json)
"""
import contextlib
import io
import json
import os
import sys
import types

import numpy as np
import scipy

REF = "/root/reference"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from make_golden_shapes import dense_cov_p  # noqa: E402
OUT = os.path.dirname(os.path.abspath(__file__))

np.float = float  # removed alias used at samplers.py:33, :359-360 (Python-2/NumPy<1.24 era)
np.int = int      # removed alias used at samplers.py:399


def _load(name, path):
    from lib2to3 import refactor
    src = open(path).read() + "\n"
    tool = refactor.RefactoringTool(["lib2to3.fixes.fix_print", "lib2to3.fixes.fix_xrange"])
    src = str(tool.refactor_string(src, name))
    src = src.replace("n = L_chain/2", "n = L_chain//2")  # utils.py:102 (Py2 int division)
    mod = types.ModuleType(name)
    exec(compile(src, path, "exec"), mod.__dict__)
    sys.modules[name] = mod
    return mod


import matplotlib  # noqa: E402
matplotlib.use("Agg")
ref_utils = _load("utils", os.path.join(REF, "utils.py"))
ref_samplers = _load("samplers", os.path.join(REF, "samplers.py"))

_orig = dict(mvn=np.random.multivariate_normal, randint=np.random.randint, random=np.random.random)


class Recorder:
    """Pass-through recorder of the legacy global RNG calls, in call order."""

    def __init__(self):
        self.log = []

    def __enter__(self):
        rec = self.log

        def mvn(*a, **k):
            v = _orig["mvn"](*a, **k)
            rec.append(("mvn", np.array(v, dtype=np.float64)))
            return v

        def randint(*a, **k):
            v = _orig["randint"](*a, **k)
            rec.append(("randint", np.array(v)))
            return v

        def random(*a, **k):
            v = _orig["random"](*a, **k)
            rec.append(("random", np.array(v, dtype=np.float64)))
            return v

        np.random.multivariate_normal = mvn
        np.random.randint = randint
        np.random.random = random
        return self

    def __exit__(self, *exc):
        np.random.multivariate_normal = _orig["mvn"]
        np.random.randint = _orig["randint"]
        np.random.random = _orig["random"]


def mvn_target(D, rho, diag=None, q0=None):
    """Target of case*-script.py:26-49: Sigma = (1-rho) I + rho 11^T (or a given diagonal)."""
    if diag is not None:
        cov0 = np.diag(np.asarray(diag, dtype=np.float64))
    else:
        cov0 = np.diag(np.ones(D)) * (1 - rho)
        cov0 += rho
    q0 = np.zeros(D) if q0 is None else np.asarray(q0, dtype=np.float64)
    inv_cov0 = np.linalg.inv(cov0)

    def V(q):
        return -ref_utils.normal_lnL(q, q0, cov0)

    def dVdq(q):
        return np.dot(inv_cov0, (q - q0))

    return q0, cov0, inv_cov0, V, dVdq


def run_random(name, D, rho, Nchain, Niter, wu, thin, L_low, L_high, dt, seed,
               start_scale=2.0, diag=None, q0=None, cov_p=None, case2_override=False, n_save=0):
    q0_, cov0, inv_cov0, V, dVdq = mvn_target(D, rho, diag, q0)
    np.random.seed(seed)
    with Recorder() as rec:
        q_start = ref_utils.start_pts(q0_, np.diag(np.ones(D)) * start_scale, Nchain)
        if case2_override:  # case2-script.py:59-61
            q_start[0, :] = 0
            q_start[0, 0] = 1000
            q_start[0, 1] = -750
        h = ref_samplers.HMC_sampler(D, V, dVdq, Niter=Niter, Nchain=Nchain, sampler_type="Random",
                                     L_low=L_low, L_high=L_high, dt=dt, thin_rate=thin,
                                     warm_up_num=wu, cov_p=cov_p)
        with contextlib.redirect_stdout(io.StringIO()):
            h.gen_sample(q_start, N_save_chain0=n_save, verbose=False)
            h.compute_convergence_stats()
    log = rec.log
    # Split the log: [mvn start] then per chain [mvn p0] + Niter x [mvn, randint, random]
    assert log[0][0] == "mvn"
    pos = 1
    p0 = np.zeros((Nchain, D)); P = np.zeros((Nchain, Niter, D))
    Ls = np.zeros((Nchain, Niter), np.int32); U = np.zeros((Nchain, Niter))
    for m in range(Nchain):
        assert log[pos][0] == "mvn"; p0[m] = log[pos][1].reshape(D); pos += 1
        for i in range(Niter):
            assert [log[pos + j][0] for j in range(3)] == ["mvn", "randint", "random"]
            P[m, i] = log[pos][1].reshape(D)
            Ls[m, i] = int(log[pos + 1][1].reshape(-1)[0])
            U[m, i] = float(log[pos + 2][1].reshape(-1)[0])
            pos += 3
    assert pos == len(log)
    qc = h.q_chain
    out = dict(
        q_start=q_start, p0=p0, p=P, L=Ls, u=U, lnu=np.log(U),
        q_chain=qc, E_chain=h.E_chain[:, :, 0], dE_chain=h.dE_chain[:, :, 0],
        accept_R=np.float64(h.accept_R),
        accept_R_warm_up=np.float64(np.nan if h.accept_R_warm_up is None else h.accept_R_warm_up),
        N_total_steps=np.int64(h.N_total_steps), n_leapfrog=np.int64(Ls.sum()),
        R_q=h.R_q, n_eff_q=h.n_eff_q,
        mean=np.array([np.mean(qc[:, 1:, i]) for i in range(D)]),   # samplers.py:246
        std=np.array([np.std(qc[:, 1:, i]) for i in range(D)]),     # samplers.py:213
        q0=q0_, cov0=cov0, inv_cov0=inv_cov0,
        cov_p=h.cov_p, dt=np.asarray(dt, dtype=np.float64),
    )
    if n_save > 0:
        out["decision_chain"] = h.decision_chain[:, 0].astype(np.int32)
        out["phi_q_len"] = np.array([x.shape[0] for x in h.phi_q], np.int32)
        out["phi_q_flat"] = np.concatenate(h.phi_q, axis=0)
    meta = dict(name=name, sampler="Random", D=D, rho=rho, Nchain=Nchain, Niter=Niter, warm_up=wu,
                thin=thin, L_low=L_low, L_high=L_high, seed=seed, start_scale=start_scale,
                diag=None if diag is None else list(map(float, diag)),
                case2_override=case2_override, n_save=n_save,
                numpy=np.__version__, scipy=scipy.__version__)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), meta=json.dumps(meta), **out)
    print(name, "accept", h.accept_R, "wu", h.accept_R_warm_up, "N_total", h.N_total_steps,
          "lf", Ls.sum())


def run_nuts(name, D, rho, Nchain, Niter, wu, thin, dt, d_max, seed):
    q0_, cov0, inv_cov0, V, dVdq = mvn_target(D, rho)
    np.random.seed(seed)
    with Recorder() as rec:
        q_start = ref_utils.start_pts(q0_, np.diag(np.ones(D)) * 2, Nchain)
        h = ref_samplers.HMC_sampler(D, V, dVdq, Niter=Niter, Nchain=Nchain, sampler_type="NUTS",
                                     dt=dt, thin_rate=thin, warm_up_num=wu, d_max=d_max)
        n_lf = [0]
        lf = h.leap_frog

        def counting_lf(p, q):
            n_lf[0] += 1
            return lf(p, q)
        h.leap_frog = counting_lf
        with contextlib.redirect_stdout(io.StringIO()) as so:
            h.gen_sample(q_start, N_save_chain0=0, verbose=False)
            h.compute_convergence_stats()
    log = rec.log
    assert log[0][0] == "mvn"
    pos = 1
    p0 = np.zeros((Nchain, D)); P = np.zeros((Nchain, Niter, D))
    tape, tape_off = [], []   # per chain: flat draws (randint -> 0/1, random -> u) and per-iteration offsets
    for m in range(Nchain):
        assert log[pos][0] == "mvn"; p0[m] = log[pos][1].reshape(D); pos += 1
        t, off = [], [0]
        for i in range(Niter):
            assert log[pos][0] == "mvn"; P[m, i] = log[pos][1].reshape(D); pos += 1
            while pos < len(log) and log[pos][0] != "mvn":
                t.append(float(log[pos][1].reshape(-1)[0])); pos += 1
            off.append(len(t))
        tape.append(np.array(t)); tape_off.append(np.array(off, np.int64))
    assert pos == len(log)
    tmax = max(len(t) for t in tape)
    tape_arr = np.full((Nchain, tmax), np.nan)
    for m in range(Nchain):
        tape_arr[m, :len(tape[m])] = tape[m]
    qc = h.q_chain
    np.savez_compressed(
        os.path.join(OUT, name + ".npz"),
        meta=json.dumps(dict(name=name, sampler="NUTS", D=D, rho=rho, Nchain=Nchain, Niter=Niter,
                             warm_up=wu, thin=thin, dt=dt, d_max=d_max, seed=seed,
                             unstable_msgs=so.getvalue().count("instability"),
                             numpy=np.__version__, scipy=scipy.__version__)),
        q_start=q_start, p0=p0, p=P, tape=tape_arr, tape_off=np.stack(tape_off),
        q_chain=qc, E_chain=h.E_chain[:, :, 0], dE_chain=h.dE_chain[:, :, 0],
        N_total_steps=np.int64(h.N_total_steps), n_leapfrog=np.int64(n_lf[0]),
        R_q=h.R_q, n_eff_q=h.n_eff_q, q0=q0_, cov0=cov0, inv_cov0=inv_cov0)
    print(name, "N_total", h.N_total_steps, "lf", n_lf[0], "tape", [len(t) for t in tape])


def run_leapfrog_vectors():
    """F4: single leap_frog / E calls of the reference (samplers.py:811-839)."""
    rng = np.random.RandomState(123)
    out = {}
    cases = [("unit100", 100, 0.0, None, 0.1), ("dense100", 100, 0.95, None, 0.1),
             ("diag10_vecdt", 10, 0.0, np.linspace(0.5, 3.0, 10), np.linspace(0.05, 0.2, 10))]
    for tag, D, rho, diag, dt in cases:
        q0_ = rng.randn(D) * 0.3 if diag is not None else None
        q0_, cov0, inv_cov0, V, dVdq = mvn_target(D, rho, diag, q0_)
        cov_p = np.diag(np.linspace(0.8, 1.5, D)) if diag is not None else None
        h = ref_samplers.HMC_sampler(D, V, dVdq, Niter=1, Nchain=2, sampler_type="Random",
                                     L_low=1, L_high=2, dt=dt, cov_p=cov_p)
        P = rng.randn(8, D); Q = rng.randn(8, D) * 1.5
        Pn = np.zeros_like(P); Qn = np.zeros_like(Q); E = np.zeros(8)
        for k in range(8):
            Pn[k], Qn[k] = h.leap_frog(P[k], Q[k])
            E[k] = h.E(Q[k], P[k])
        out.update({f"{tag}_p": P, f"{tag}_q": Q, f"{tag}_pn": Pn, f"{tag}_qn": Qn, f"{tag}_E": E,
                    f"{tag}_q0": q0_, f"{tag}_cov0": cov0, f"{tag}_inv_cov0": inv_cov0,
                    f"{tag}_cov_p": h.cov_p, f"{tag}_dt": np.asarray(dt, np.float64)})
    np.savez_compressed(os.path.join(OUT, "f4_leapfrog.npz"), **out)
    print("f4_leapfrog done")


def run_convergence():
    """F5: convergence_stats (utils.py:77-179) on synthetic AR(1) chains."""
    rng = np.random.RandomState(7)
    out = {}
    shapes = [("a", 4, 201, 3, 0.0), ("b", 4, 200, 3, 0.5), ("c", 2, 51, 2, 0.95),
              ("d", 10, 1000, 5, 0.9), ("e", 3, 9, 2, 0.3), ("f", 6, 400, 4, -0.4)]
    for tag, N, T, D, phi in shapes:
        x = np.zeros((N, T, D))
        x[:, 0] = rng.randn(N, D) * 2
        for t in range(1, T):
            x[:, t] = phi * x[:, t - 1] + rng.randn(N, D)
        R, neff = ref_utils.convergence_stats(x, warm_up_num=0, thin_rate=1)
        out[f"{tag}_x"] = x; out[f"{tag}_R"] = R; out[f"{tag}_neff"] = neff
        R2, neff2 = ref_utils.convergence_stats(x, thin_rate=5, warm_up_num=3)  # defaults path
        out[f"{tag}_R_thin5"] = R2; out[f"{tag}_neff_thin5"] = neff2
    np.savez_compressed(os.path.join(OUT, "f5_convergence.npz"), **out)
    print("f5_convergence done")


def run_tree_tables():
    """F7: NUTS bookkeeping known answers (utils.py:246-283, :367-385, README:287-365)."""
    cps = {}
    rel = {}
    for m in range(2, 129, 2):
        c = [int(v) for v in ref_utils.check_points(m)]
        cps[m] = c
        rel[m] = [bool(ref_utils.release_fast(m, l)) for l in c]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        ref_utils.test_NUTS_binary_tree_flatten()
    json.dump(dict(check_points=cps, release=rel, flatten_print=buf.getvalue().splitlines()),
              open(os.path.join(OUT, "f7_tree.json"), "w"), indent=0)
    print("f7_tree done")


if __name__ == "__main__":
    run_random("f1_case1a", D=2, rho=0.0, Nchain=10, Niter=2000, wu=1000, thin=1,
               L_low=5, L_high=20, dt=0.1, seed=0, n_save=100)
    run_random("f2_case1c_small", D=100, rho=0.0, Nchain=3, Niter=200, wu=50, thin=1,
               L_low=5, L_high=20, dt=0.1, seed=1)
    run_random("f3_case3c_small", D=100, rho=0.95, Nchain=3, Niter=150, wu=50, thin=1,
               L_low=5, L_high=20, dt=0.1, seed=2)
    run_random("f3b_case3a", D=2, rho=0.95, Nchain=4, Niter=400, wu=200, thin=1,
               L_low=5, L_high=20, dt=0.1, seed=3)
    run_random("f8_diag_thin_vecdt", D=10, rho=0.0, Nchain=4, Niter=100, wu=7, thin=3,
               L_low=3, L_high=9, dt=np.linspace(0.05, 0.15, 10), seed=4,
               diag=np.linspace(0.5, 3.0, 10), q0=np.linspace(-1, 1, 10),
               cov_p=np.diag(np.linspace(0.8, 1.5, 10)))
    run_random("f9_wu0_thin2", D=5, rho=0.0, Nchain=3, Niter=50, wu=0, thin=2,
               L_low=5, L_high=20, dt=0.1, seed=5)
    run_random("f10_case2a", D=2, rho=0.0, Nchain=4, Niter=300, wu=100, thin=1,
               L_low=5, L_high=20, dt=0.1, seed=6, start_scale=100.0, case2_override=True, n_save=20)
    run_random("f11_case5_unstable", D=10, rho=0.999, Nchain=3, Niter=120, wu=40, thin=1,
               L_low=5, L_high=20, dt=0.1, seed=8)
    run_random("f12_dense_covp", D=12, rho=0.6, Nchain=3, Niter=90, wu=30, thin=1,
               L_low=5, L_high=20, dt=0.1, seed=12, cov_p=dense_cov_p(12))
    run_nuts("f6_nuts_dense100", D=100, rho=0.95, Nchain=2, Niter=12, wu=4, thin=1, dt=0.1,
             d_max=12, seed=9)
    run_leapfrog_vectors()
    run_convergence()
    run_tree_tables()
