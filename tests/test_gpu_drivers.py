"""The Python-3 case driver (drivers/cases.py) end to end: case 1a with np.random.seed(0)
reproduces the reference run recorded in tests/golden/f1_case1a.npz (the reference's
case1-script.py case 1a, same seed): bit-identical q_chain, acceptance, N_total_steps, and
R-hat / ESS within the 1e-6 contract."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT, load_golden

sys.path.insert(0, os.path.join(ROOT, "drivers"))


@pytest.mark.gpu
def test_case1a_reproduces_reference():
    from cases import run_case
    g = load_golden("f1_case1a.npz")
    h = run_case("1a", seed=0, rng="replay", fp_mode="exact", verbose=False)
    np.testing.assert_array_equal(h.q_chain, g["q_chain"])
    assert h.accept_R == float(g["accept_R"])
    assert h.accept_R_warm_up == float(g["accept_R_warm_up"])
    assert h.N_total_steps == int(g["N_total_steps"])
    np.testing.assert_allclose(h.R_q, g["R_q"], rtol=1e-6)
    np.testing.assert_allclose(h.n_eff_q, g["n_eff_q"], rtol=1e-6)
    assert len(h.phi_q) == 100


@pytest.mark.gpu
def test_case1a_driver_ends_with_reference_figures(tmp_path):
    """The driver run ends the way case1-script.py:66-67 does: plot_samples(savefig) and
    make_movie on the sampler the GPU filled.  The figure's numbers (plots.sample_summary) are the
    reference's F1 anchors (per-dim mean/std by the reference's own expressions, samplers.py:213,
    :246), and the movie's first slides follow the GPU's chain-0 capture."""
    from cases import run_case, title_prefix
    from hmc_amd import plots
    g = load_golden("f1_case1a.npz")
    h = run_case("1a", seed=0, rng="replay", fp_mode="exact", verbose=False, plots=True, out_dir=str(tmp_path),
                 movie_frames=3, movie_dpi=40)
    S = h.plot_summary
    assert np.array_equal(S["q_mean"], g["mean"]) and np.array_equal(S["q_std"], g["std"])
    assert np.allclose(S["q_std"], [1.01934971, 0.98600590], atol=5e-9)          # SURVEY §8(c) F1 anchors
    assert S["stats"]["N_samples"] == 10 * 1001
    title = title_prefix("1a", str(tmp_path))
    assert title.endswith(os.path.join("case1", "case1a"))
    png = title + "-samples-D2-Nchain10-Niter2000-Warm1000-Thin1.png"
    assert S["fname"] == png and os.path.getsize(png) > 10000
    assert h.movie_files == ["%s-slide-%d.png" % (title, i) for i in range(3)]
    assert all(os.path.getsize(f) > 1000 for f in h.movie_files)
    frames = plots.movie_frames(h.phi_q, h.decision_chain)
    assert frames[0] == (0, 1, int(g["decision_chain"][0]))
    assert len(frames) == int(g["phi_q_len"].sum())


def test_case_table_covers_reference_scripts():
    from cases import CASES
    assert {"1a", "1b", "1c", "2a", "2b", "2c", "3a", "3b", "3c", "3-2", "4a", "4b", "4c", "5a", "5b", "5c"} <= set(CASES)
