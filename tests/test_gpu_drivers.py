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


def test_case_table_covers_reference_scripts():
    from cases import CASES
    assert {"1a", "1b", "1c", "2a", "2b", "2c", "3a", "3b", "3c", "3-2", "4a", "4b", "4c", "5a", "5b", "5c"} <= set(CASES)
