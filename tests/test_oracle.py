"""Pin the CPU oracle (oracle/hmc_oracle.py) against the reference's own outputs.

The fixtures in tests/golden/ were produced by running the reference
(/root/reference samplers.py + utils.py, translated in memory) — see
tests/golden/make_golden.py.  With the recorded random streams replayed, the
oracle must reproduce every output BIT-EXACTLY (same NumPy/SciPy operations in
the same order).  CPU only.
"""
import numpy as np
import pytest

from conftest import load_golden
from oracle import hmc_oracle as O

RANDOM_FIXTURES = ["f1_case1a.npz", "f2_case1c_small.npz", "f3_case3c_small.npz", "f3b_case3a.npz",
                   "f8_diag_thin_vecdt.npz", "f9_wu0_thin2.npz", "f10_case2a.npz",
                   "f11_case5_unstable.npz", "f12_dense_covp.npz"]


def _core(g):
    dt = g["dt"]
    dt = float(dt) if dt.ndim == 0 else dt
    return O.HMCCore(O.MVNTarget(g["q0"], g["cov0"]), dt, g["cov_p"])


@pytest.mark.parametrize("fx", RANDOM_FIXTURES)
def test_random_engine_replay_bitexact(fx):
    g = load_golden(fx)
    m = g["meta"]
    out = O.gen_sample_random(_core(g), g["q_start"], m["Nchain"], m["Niter"], m["warm_up"],
                              m["thin"], m["L_low"], m["L_high"],
                              O.ReplayDraws(g["p0"], g["p"], g["L"], g["lnu"]),
                              n_save_chain0=m["n_save"])
    assert np.array_equal(out["q_chain"], g["q_chain"])
    assert np.array_equal(out["E_chain"], g["E_chain"])
    assert np.array_equal(out["dE_chain"], g["dE_chain"])
    assert out["accept_R"] == g["accept_R"]
    if m["warm_up"] > 0:
        assert out["accept_R_warm_up"] == g["accept_R_warm_up"]
    else:
        assert out["accept_R_warm_up"] is None and np.isnan(g["accept_R_warm_up"])
    assert out["N_total_steps"] == int(g["N_total_steps"])
    assert out["n_leapfrog"] == int(g["n_leapfrog"])
    if m["n_save"]:
        assert np.array_equal(out["decision_chain"], g["decision_chain"])
        assert np.array_equal(np.concatenate(out["phi_q"]), g["phi_q_flat"])
    R, neff = O.convergence_stats(out["q_chain"][:, 1:, :], warm_up_num=0, thin_rate=1)
    assert np.array_equal(R, g["R_q"]) and np.array_equal(neff, g["n_eff_q"])
    mean, std = O.per_dim_mean_std(out["q_chain"])
    assert np.array_equal(mean, g["mean"]) and np.array_equal(std, g["std"])


def test_case1a_anchors():
    """SURVEY.md §8(c) F1 anchors observed from the reference (seed 0)."""
    g = load_golden("f1_case1a.npz")
    assert abs(float(g["accept_R_warm_up"]) - 0.997700) < 5e-7
    assert abs(float(g["accept_R"]) - 0.998801) < 5e-7
    assert int(g["N_total_steps"]) == 6556744 and int(g["n_leapfrog"]) == 240327
    np.testing.assert_allclose(g["R_q"], [1.00121354, 1.00087536], rtol=1e-8)
    np.testing.assert_allclose(g["std"], [1.01934971, 0.98600590], rtol=1e-8)


@pytest.mark.parametrize("fx", ["f3b_case3a.npz", "f9_wu0_thin2.npz"])
def test_random_engine_live_rng_order(fx):
    """Live mode (global legacy np.random, reference call order Q7) regenerates the
    recorded streams and outputs from the seed alone."""
    g = load_golden(fx)
    m = g["meta"]
    np.random.seed(m["seed"])
    D = m["D"]
    q_start = O.start_pts(np.zeros(D), np.diag(np.ones(D)) * m["start_scale"], m["Nchain"])
    assert np.array_equal(q_start, g["q_start"])
    core = _core(g)
    out = O.gen_sample_random(core, q_start, m["Nchain"], m["Niter"], m["warm_up"], m["thin"],
                              m["L_low"], m["L_high"], O.LiveDraws(D, core.cov_p))
    assert np.array_equal(out["q_chain"], g["q_chain"])
    assert np.array_equal(out["E_chain"], g["E_chain"])


def test_identity_mvn_equals_standard_normal():
    """Q7: multivariate_normal(0, I) consumes the stream exactly like standard_normal(D)
    and returns the same values bitwise (lets replay streams be drawn cheaply)."""
    for D in (2, 10, 100):
        np.random.seed(11)
        a = np.stack([np.random.multivariate_normal(np.zeros(D), np.eye(D), size=1)[0]
                      for _ in range(5)])
        np.random.seed(11)
        b = np.stack([np.random.standard_normal(D) for _ in range(5)])
        assert np.array_equal(a, b)


def test_nuts_replay_bitexact():
    g = load_golden("f6_nuts_dense100.npz")
    m = g["meta"]
    core = O.HMCCore(O.MVNTarget(g["q0"], g["cov0"]), m["dt"])
    tape = g["tape"]
    out = O.gen_sample_nuts(core, g["q_start"], m["Nchain"], m["Niter"], m["warm_up"], m["thin"],
                            m["d_max"], O.ReplayDraws(g["p0"], g["p"], tape=tape))
    assert np.array_equal(out["q_chain"], g["q_chain"])
    assert np.array_equal(out["E_chain"], g["E_chain"])
    assert np.array_equal(out["dE_chain"], g["dE_chain"])
    assert out["N_total_steps"] == int(g["N_total_steps"])
    assert out["n_leapfrog"] == int(g["n_leapfrog"])


def test_leapfrog_vectors():
    g = load_golden("f4_leapfrog.npz")
    for tag in ("unit100", "dense100", "diag10_vecdt"):
        dt = g[f"{tag}_dt"]
        core = O.HMCCore(O.MVNTarget(g[f"{tag}_q0"], g[f"{tag}_cov0"]),
                         float(dt) if dt.ndim == 0 else dt, g[f"{tag}_cov_p"])
        for k in range(g[f"{tag}_p"].shape[0]):
            pn, qn = core.leap_frog(g[f"{tag}_p"][k], g[f"{tag}_q"][k])
            assert np.array_equal(pn, g[f"{tag}_pn"][k]) and np.array_equal(qn, g[f"{tag}_qn"][k])
            assert core.E(g[f"{tag}_q"][k], g[f"{tag}_p"][k]) == g[f"{tag}_E"][k]


def test_convergence_stats_vectors():
    g = load_golden("f5_convergence.npz")
    for tag in "abcdef":
        x = g[f"{tag}_x"]
        with np.errstate(all="ignore"):
            R, neff = O.convergence_stats(x, warm_up_num=0, thin_rate=1)
            R5, neff5 = O.convergence_stats(x, thin_rate=5, warm_up_num=3)
        np.testing.assert_array_equal(R, g[f"{tag}_R"])
        np.testing.assert_array_equal(neff, g[f"{tag}_neff"])
        np.testing.assert_array_equal(R5, g[f"{tag}_R_thin5"])
        np.testing.assert_array_equal(neff5, g[f"{tag}_neff_thin5"])


def test_tree_tables_vs_reference_and_readme():
    t = load_golden("f7_tree.json")
    for m, pts in t["check_points"].items():
        m = int(m)
        assert list(O.check_points(m)) == pts
        assert [bool(O.release_fast(m, l)) for l in pts] == t["release"][str(m)]
    # README:332-358 "Check points -- examples" / "Release -- examples"
    assert list(O.check_points(8)) == [1, 5, 7]
    assert list(O.check_points(16)) == [1, 9, 13, 15]
    assert list(O.check_points(24)) == [17, 21, 23]
    assert list(O.check_points(32)) == [1, 17, 25, 29, 31]
    assert [l for l in O.check_points(16) if l > 1 and O.release_fast(16, l)] == [9, 13, 15]
    assert [l for l in O.check_points(24) if l > 1 and O.release_fast(24, l)] == [21, 23]
    # utils.test_NUTS_binary_tree_flatten printout (README:294-325 pattern), replayed
    table = [-1] * 11
    lines = []
    for m in range(2, 33):
        def line():
            return "%2d: " % m + "".join("x " if (i in table or i == 1 or i == m) else "o "
                                           for i in range(1, m + 1))
        if m % 2 == 1:
            table[O.find_next(table)] = m
            lines.append(line())
        else:
            lines.append(line())
            for l in O.check_points(m):
                s = O.retrieve_save_index(table, l)
                if l > 1 and O.release_fast(m, l):
                    table[s] = -1
    assert lines == t["flatten_print"]


def test_nuts_closed_form_save_slots():
    """hmc_nuts.hip keeps saved odd point l of a sub-tree in slot ctz(l - 1) (point 1: slot
    d_max) instead of the reference's searched table (utils.py:222-385): every point that
    check_points(m) names must still be in its slot when m is reached, for every sub-tree size
    the reference can build (d < d_max <= 15), and for trees up to 2^17 points at d_max = 30 (the
    kernels' bound: slots depend on d_max only through point 1's)."""
    from hmc_amd.utils import check_points

    def slot(l, d_max):
        return d_max if l == 1 else ((l - 1) & -(l - 1)).bit_length() - 1
    for d_max in range(1, 16):
        for d in range(d_max):
            held = {}
            for m in range(1, (1 << d) + 1):
                if m % 2:
                    assert 0 <= slot(m, d_max) <= d_max
                    held[slot(m, d_max)] = m
                else:
                    for l in check_points(m):
                        assert held.get(slot(int(l), d_max)) == int(l), (d_max, d, m, l)
    held = {}
    d_max = 30
    for m in range(1, (1 << 17) + 1):      # one pass: a tree of 2^17 points holds every smaller one's steps
        if m % 2:
            held[slot(m, d_max)] = m
        elif m & (m - 1) == 0 or m % 64 == 0 or m > (1 << 17) - 4096:
            for l in check_points(m):
                assert held.get(slot(int(l), d_max)) == int(l), (d_max, m, l)


def test_reference_nuts_drifts_with_a_mass_matrix():
    """A property of the reference the large-D NUTS tests rely on: with cov_p other than the
    identity, the reference's NUTS (Q3 leapfrog: kick by inv(cov_p).dVdq, drift by p; Q11 ratio;
    samplers.py:495-808, :831-839) does not keep N(0, Sigma), so GPU runs with a full cov_p are
    pinned by replay parity, not by a stationarity check.  Oracle on np.random draws, D = 8."""
    import make_golden_shapes as S
    np.random.seed(1)
    D, N = 8, 600
    cov = O.mvn_cov(D, 0.6)
    qs = np.random.standard_normal((N, D)) @ np.linalg.cholesky(cov).T
    var = {}
    for name, cp in (("full", S.dense_cov_p(D)), ("none", np.eye(D))):
        np.random.seed(2)
        ref = O.gen_sample_nuts(O.HMCCore(O.MVNTarget(np.zeros(D), cov), 0.2, cp), qs, N, 3, 1, 1, 8,
                                O.LiveDraws(D, cp), on_dmax="break")
        var[name] = ref["q_chain"][:, -1, :].var(axis=0).mean()
    noise = 6 * np.sqrt(2 / (N * D))
    assert var["full"] > 1 + noise + 0.1
    assert abs(var["none"] - 1) < noise + 0.05
