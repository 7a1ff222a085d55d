"""INTEGRATION.md §2's raw ctypes binding, as a maintainer would paste it next to samplers.py.

The struct definitions and argtypes are taken from the document's first code block (executed as
written, so the document cannot drift from include/hmc.h without failing here), not from
hmc_amd/_lib.py.  CPU: every struct's fields, offsets and size equal the maintained binding's
(which tests/test_abi.py checks against the header).  GPU: hmc_chain_init + hmc_nuts_iters_ws
with a full cov_p (minv_full, kick) at D = 136 (the per-chain kernel) on replayed draws, against
the oracle's gen_sample_NUTS (samplers.py:352-356, :495-808)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STRUCTS = ["hmc_target", "hmc_kinetic", "hmc_schedule", "hmc_replay", "hmc_state"]


def _section2_blocks():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 2."):text.index("## 3.")]
    return re.findall(r"```python\n(.*?)```", sec, re.S)


def _binding(monkeypatch):
    """Namespace of INTEGRATION.md §2's first block (it loads the library by its repo-relative path)."""
    monkeypatch.chdir(ROOT)
    ns = {}
    exec(compile(_section2_blocks()[0], "INTEGRATION.md#2", "exec"), ns)
    return ns


def test_integration_blocks_present():
    blocks = _section2_blocks()
    assert len(blocks) == 3                      # the binding, the Random call, the NUTS call
    assert "hmc_nuts_iters_ws" in blocks[2] and "minv_full" in blocks[2]


def test_integration_structs_match_binding(monkeypatch):
    from hmc_amd import _lib as H
    ns = _binding(monkeypatch)
    mine = {"hmc_target": H.Target, "hmc_kinetic": H.Kinetic, "hmc_schedule": H.Schedule,
            "hmc_replay": H.Replay, "hmc_state": H.State}
    for name in STRUCTS:
        doc, lib = ns[name], mine[name]
        assert [f[0] for f in doc._fields_] == [f[0] for f in lib._fields_], name
        for (fname, ftype), (_, ltype) in zip(doc._fields_, lib._fields_):
            assert ctypes.sizeof(ftype) == ctypes.sizeof(ltype), (name, fname)
            assert getattr(doc, fname).offset == getattr(lib, fname).offset, (name, fname)
        assert ctypes.sizeof(doc) == ctypes.sizeof(lib), name
    rename = {"hmc_target": "Target", "hmc_kinetic": "Kinetic", "hmc_schedule": "Schedule",
              "hmc_replay": "Replay", "hmc_state": "State"}

    def kind(t):                                 # struct pointers by struct, scalars by C type
        s = getattr(t, "_type_", None)
        if isinstance(s, type) and issubclass(s, ctypes.Structure):
            return "P(" + rename.get(s.__name__, s.__name__) + ")"
        return t._type_ if isinstance(t._type_, str) else t.__name__
    for fn in ("hmc_chain_init", "hmc_random_iters", "hmc_nuts_iters_ws", "hmc_random_workspace_size_ex",
               "hmc_nuts_workspace_size_ex"):
        f = getattr(ns["lib"], fn)
        restype, argtypes = H.SYMBOLS[fn]
        assert [kind(t) for t in f.argtypes] == [kind(t) for t in argtypes], fn
        assert ctypes.sizeof(f.restype) == ctypes.sizeof(restype), fn


@pytest.mark.gpu
def test_integration_nuts_full_cov_p_d136_vs_oracle(monkeypatch):
    import torch
    import make_golden_shapes as GS
    from oracle import hmc_oracle as O
    ns = _binding(monkeypatch)
    lib = ns["lib"]
    hmc_target, hmc_kinetic, hmc_schedule = ns["hmc_target"], ns["hmc_kinetic"], ns["hmc_schedule"]
    hmc_replay, hmc_state = ns["hmc_replay"], ns["hmc_state"]
    D, N, Niter, wu, thin, dt, d_max = 136, 3, 5, 1, 1, 0.15, 7
    rs = np.random.RandomState(136)
    cov0, cov_p = O.mvn_cov(D, 0.6), GS.dense_cov_p(D)
    C = np.linalg.cholesky(cov_p)
    q_start = rs.standard_normal((N, D)) * 1.2
    p0 = rs.standard_normal((N, D)) @ C.T
    Pm = rs.standard_normal((N, Niter, D)) @ C.T
    tape = rs.uniform(0.0, 2.0, (N, Niter * 2 * (2 ** d_max + d_max + 2)))
    logdet_const = float(D * np.log(2 * np.pi) + np.linalg.slogdet(cov0)[1])

    class Tgt(O.MVNTarget):                      # V with the same constant the kernel is given
        def V(self, q):
            return 0.5 * (logdet_const + q @ (self.inv_cov0 @ q))
    ref = O.gen_sample_nuts(O.HMCCore(Tgt(np.zeros(D), cov0), dt, cov_p), q_start, N, Niter, wu, thin, d_max,
                            O.ReplayDraws(p0, Pm, tape=tape.copy()), on_dmax="break")

    def dev(a):
        return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device="cuda")
    Minv = np.linalg.inv(cov_p)                                    # samplers.py:356
    prec, minv_full, chol_t = dev(np.linalg.inv(cov0)), dev(Minv), dev(C.T)
    kick = dev(Minv @ np.linalg.inv(cov0))                         # inv_cov_p . P (:835-837)
    Lc = 1 + (Niter - wu) // thin
    q, Ep = torch.empty((N, D), dtype=torch.float64, device="cuda"), torch.empty(N, dtype=torch.float64, device="cuda")
    qc = torch.zeros((N, Lc, D), dtype=torch.float64, device="cuda")
    Ec, dEc = torch.zeros((N, Lc), dtype=torch.float64, device="cuda"), torch.zeros((N, Lc), dtype=torch.float64, device="cuda")
    cnt = torch.zeros((4096, 9), dtype=torch.int64, device="cuda")
    qs, p0d, Pd, taped = dev(q_start), dev(p0), dev(Pm), dev(tape)
    T = hmc_target(D, 1, None, prec.data_ptr(), logdet_const)
    K = hmc_kinetic(None, None, None, dt, minv_full.data_ptr(), chol_t.data_ptr(), kick.data_ptr())
    R = hmc_replay(p0d.data_ptr(), Pd.data_ptr(), None, None, taped.data_ptr(), tape.shape[1])
    order = torch.zeros(max(lib.hmc_random_workspace_size_ex(T, K, N), 1), dtype=torch.uint8, device="cuda")
    st = hmc_state(q.data_ptr(), Ep.data_ptr(), qc.data_ptr(), Ec.data_ptr(), dEc.data_ptr(), cnt.data_ptr(),
                   None, None, None, 0, 0, 0, 0, order.data_ptr())
    nbytes = lib.hmc_nuts_workspace_size_ex(D, N, d_max, Niter, 0)
    assert nbytes > 0
    ws = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream

    def sched(i0, i1):
        return hmc_schedule(N, 0, Niter, wu, thin, Lc, 0, 0, i0, i1, 0, 0, d_max, 1, 0)   # REPLAY, EXACT, break
    assert lib.hmc_chain_init(T, K, sched(1, 1), R, qs.data_ptr(), st, stream) == 0, lib.hmc_last_error()
    for i0, i1 in ((1, 3), (3, Niter + 1)):                        # two calls: tape cursors persist
        assert lib.hmc_nuts_iters_ws(T, K, sched(i0, i1), R, st, ws.data_ptr(), nbytes, stream) == 0, \
            lib.hmc_last_error()
    # a workspace one byte short is refused before anything runs
    assert lib.hmc_nuts_iters_ws(T, K, sched(1, 2), R, st, ws.data_ptr(), nbytes - 1, stream) == 1
    torch.cuda.synchronize()
    c = cnt.sum(0).cpu().numpy()
    assert int(c[4]) == 0                                          # HMC_CNT_OOB_REJECT
    assert int(c[8]) == 0                                          # HMC_CNT_HANDOFF_GIVEUP
    assert int(c[2]) == ref["n_leapfrog"]                          # HMC_CNT_LEAPFROG
    assert int(c[5]) == ref["n_unstable"]                          # HMC_CNT_UNSTABLE
    np.testing.assert_allclose(qc.cpu().numpy(), ref["q_chain"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(Ec.cpu().numpy(), ref["E_chain"], rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(dEc.cpu().numpy(), ref["dE_chain"], rtol=1e-8, atol=1e-9)
