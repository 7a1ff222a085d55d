"""plot_samples / make_movie (samplers.py:67-291, :843-924) on sampler results, CPU only.

The figure's numbers come from hmc_amd.plots.sample_summary; the per-dimension mean and
std it draws must equal the reference's own F1 anchors (tests/golden/f1_case1a.npz,
computed by the reference's expressions at samplers.py:213/:246), and the movie's frame
list must follow the reference's capture (phi_q, decision_chain)."""
import types

import numpy as np
import pytest

from conftest import load_golden
from hmc_amd import plots


def _f1_sampler():
    g = load_golden("f1_case1a.npz")
    m = g["meta"]
    lens = g["phi_q_len"]
    phi = np.split(g["phi_q_flat"], np.cumsum(lens)[:-1])
    s = types.SimpleNamespace(
        D=2, Nchain=m["Nchain"], Niter=m["Niter"], warm_up_num=m["warm_up"], thin_rate=m["thin"],
        L_chain=g["q_chain"].shape[1], q_chain=g["q_chain"], E_chain=g["E_chain"][:, :, None],
        dE_chain=g["dE_chain"][:, :, None], R_q=g["R_q"], n_eff_q=g["n_eff_q"],
        accept_R=float(g["accept_R"]), accept_R_warm_up=float(g["accept_R_warm_up"]), dt_total=1.0,
        N_total_steps=int(g["N_total_steps"]), sampler_type="Random", phi_q=phi,
        decision_chain=g["decision_chain"][:, None])
    return g, s


def test_summary_matches_reference_anchors():
    g, s = _f1_sampler()
    S = plots.sample_summary(s, q0=g["q0"], cov0=g["cov0"])
    assert np.array_equal(S["q_mean"], g["mean"])
    assert np.array_equal(S["q_std"], g["std"])
    # SURVEY §8(c) F1 anchors
    assert np.allclose(S["q_mean"], [0.00327455, 0.01009606], atol=5e-9)
    assert np.allclose(S["q_std"], [1.01934971, 0.98600590], atol=5e-9)
    assert np.array_equal(S["bias"], g["mean"] - g["q0"])
    assert S["stats"]["N_samples"] == 10 * 1001
    assert S["stats"]["steps_per_es_median"] == int(g["N_total_steps"]) / np.median(g["n_eff_q"])
    # 95%-range widened 2.5x (samplers.py:93-116)
    q1 = g["q_chain"][:, :, 0].ravel()
    hi, lo = np.percentile(q1, 97.5), np.percentile(q1, 2.5)
    assert np.isclose(S["q1_max"] - S["q1_min"], 2.5 * (hi - lo))
    assert np.isclose(S["dq1"], 2.5 * (hi - lo) / 100.)


def test_plot_samples_writes_png(tmp_path):
    g, s = _f1_sampler()
    S = plots.plot_samples(s, str(tmp_path / "case1a"), savefig=True, q0=g["q0"], cov0=g["cov0"])
    fn = tmp_path / "case1a-samples-D2-Nchain10-Niter2000-Warm1000-Thin1.png"
    assert S["fname"] == str(fn) and fn.stat().st_size > 10000
    assert S["stats_text"][0] == "RA before warm-up: %.3f" % g["accept_R_warm_up"]


def test_cov_ellipse_axes():
    w, h, ang = plots.cov_ellipse(np.diag([4.0, 1.0]), nsig=1)
    r = np.sqrt(2.2957489)   # chi2.ppf(0.6827, 2)
    assert np.isclose(w, 2 * r, rtol=1e-6) and np.isclose(h, 4 * r, rtol=1e-6)
    with pytest.raises(ValueError):
        plots.cov_ellipse(np.eye(2))


def test_make_movie_frames(tmp_path):
    g, s = _f1_sampler()
    frames = plots.movie_frames(s.phi_q, s.decision_chain)
    assert len(frames) == int(g["phi_q_len"].sum())
    assert frames[0] == (0, 1, int(g["decision_chain"][0]))
    names = plots.make_movie(s, str(tmp_path / "mv"), q0=g["q0"], cov0=g["cov0"], max_frames=3, dpi=40)
    assert [n.rsplit("-", 1)[1] for n in names] == ["0.png", "1.png", "2.png"]
