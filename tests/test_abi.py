"""C-ABI boundary checks that need no GPU: libhmc.so loads, exports every function
include/hmc.h declares, the ctypes struct mirrors match the C layouts, and every entry that takes
caller-sized device scratch refuses (HMC_EINVAL, before any launch) a buffer recorded as too small
through its sized form or hmc_workspace_register (round 6)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "hmc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(hmc_[a-z_0-9]+)\s*\(", src, flags=re.M)))


def test_header_declares_entry_points():
    names = _declared()
    for must in ("hmc_chain_init", "hmc_random_iters", "hmc_leapfrog", "hmc_energy", "hmc_split_moments",
                 "hmc_variogram", "hmc_rowsum"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from hmc_amd import _lib
    L = _lib.lib()
    for name in _declared():
        assert hasattr(L, name), name
    assert set(_declared()) == set(_lib.SYMBOLS), "ctypes SYMBOLS out of sync with include/hmc.h"
    assert L.hmc_version().startswith(b"hmc_amd")


def test_struct_layouts():
    from hmc_amd import _lib as H
    # sizes follow from the C declarations (x86-64 SysV alignment)
    assert ctypes.sizeof(H.Target) == 32
    assert ctypes.sizeof(H.Kinetic) == 56
    assert ctypes.sizeof(H.Schedule) == 8 + 8 + 12 * 4 + 8
    assert ctypes.sizeof(H.Replay) == 48
    assert ctypes.sizeof(H.State) == 9 * 8 + 8 + 2 * 8 + 8


def test_counter_slots_match_header():
    """Every HMC_CNT_* slot of include/hmc.h has its mirror in _lib (one meaning per slot: the NUTS
    hand-off give-ups have their own slot, HMC_CNT_HANDOFF_GIVEUP, not HMC_CNT_ACCEPT's)."""
    from hmc_amd import _lib as H
    src = open(os.path.join(ROOT, "include", "hmc.h")).read()
    slots = {k: int(v) for k, v in re.findall(r"HMC_CNT_(\w+)\s*=\s*(\d+)", src)}
    assert slots, "no counter slots found"
    for k, v in slots.items():
        assert getattr(H, "CNT_" + k) == v, k
    assert sorted(slots.values()) == list(range(len(slots)))
    assert int(re.search(r"HMC_NCOUNTERS\s*=\s*(\d+)", src).group(1)) == H.NCOUNTERS == len(slots)
    assert int(re.search(r"HMC_COUNTER_SLOTS\s*=\s*(\d+)", src).group(1)) == H.COUNTER_SLOTS


def test_invalid_arguments_map_to_reference_exceptions():
    """Validation runs on the host before any HIP call: the reference's asserts become
    AssertionError via hmc_status HMC_EINVAL (samplers.py:331-348)."""
    from hmc_amd import _lib as H
    L = H.lib()
    T = H.Target(0, 0, None, None, 0.0)          # D = 0 -> EINVAL
    K = H.Kinetic(None, None, None, 0.1)
    S = H.Schedule(4, 0, 10, 0, 1, 11, 5, 20, 1, 11, 1, 0, 10, 0, 0)
    st = H.State()
    with pytest.raises(AssertionError):
        H.check(L.hmc_random_iters(T, K, S, None, st, None), "x")
    T.D = 3
    S.L_chain = 7                                 # wrong L_chain
    with pytest.raises(AssertionError):
        H.check(L.hmc_random_iters(T, K, S, None, st, None), "x")
    S.L_chain = 11
    S.L_high = 5                                  # L_low >= L_high (randint raises)
    with pytest.raises(AssertionError):
        H.check(L.hmc_random_iters(T, K, S, None, st, None), "x")


def test_no_cpu_fallback_when_library_missing(tmp_path, monkeypatch):
    import importlib
    from hmc_amd import _lib as H
    monkeypatch.setattr(H, "_lib", None)
    monkeypatch.setattr(H, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(RuntimeError, match="libhmc.so not found"):
        H.lib()
    importlib.reload(H)


def test_random_workspace_size_query(monkeypatch):
    """hmc_random_workspace_size: no scratch for diagonal targets; dense targets take an int32
    chain order + two 256-bin histograms and the per-chain gradient cache (host-only query)."""
    from hmc_amd import _lib as H
    monkeypatch.setattr(H, "_lib", None)     # argtypes bound to this module's structure classes
    L = H.lib()
    assert L.hmc_random_workspace_size(ctypes.byref(H.Target(100, H.HMC_TARGET_DIAG, None, None, 0.0)), 1000) == 0
    assert L.hmc_random_workspace_size(ctypes.byref(H.Target(2048, H.HMC_TARGET_DIAG, None, None, 0.0)), 1000) == 0
    # int32 tile order + histograms, 16-byte aligned, a 16-byte validity word, the [n][D] gradient cache
    assert L.hmc_random_workspace_size(ctypes.byref(H.Target(100, H.HMC_TARGET_DENSE, None, None, 0.0)), 1000) == \
        (1000 + 512) * 4 + 16 + 1000 * 100 * 8
    assert L.hmc_random_workspace_size(None, 1000) == 0
    # large D (hmc_big.hip): p, q copy (+ gradient and its copy for dense) [n][D] and three [n] arrays
    assert L.hmc_random_workspace_size(ctypes.byref(H.Target(3000, H.HMC_TARGET_DIAG, None, None, 0.0)), 1000) == \
        2 * 1000 * 3000 * 8 + 3 * 8192
    assert L.hmc_random_workspace_size(ctypes.byref(H.Target(200, H.HMC_TARGET_DENSE, None, None, 0.0)), 1000) == \
        6 * 1000 * 200 * 8 + 3 * 8192   # p, qi, g, gi + the full-cov_p products kv, u
    # sized for the kinetic part: without a full cov_p no kv, u (advisor r04)
    diag_k = H.Kinetic(None, None, None, 0.1, None, None, None)
    full_k = H.Kinetic(None, None, None, 0.1, 1, 1, 1)             # any non-NULL minv_full
    t200 = ctypes.byref(H.Target(200, H.HMC_TARGET_DENSE, None, None, 0.0))
    assert L.hmc_random_workspace_size_ex(t200, ctypes.byref(diag_k), 1000) == 4 * 1000 * 200 * 8 + 3 * 8192
    assert L.hmc_random_workspace_size_ex(t200, ctypes.byref(full_k), 1000) == 6 * 1000 * 200 * 8 + 3 * 8192
    assert L.hmc_random_workspace_size_ex(ctypes.byref(H.Target(100, H.HMC_TARGET_DENSE, None, None, 0.0)),
                                          ctypes.byref(diag_k), 1000) == (1000 + 512) * 4 + 16 + 1000 * 100 * 8


def test_nuts_workspace_size_query(monkeypatch):
    """hmc_nuts_workspace_size(_ex) (host-only query): the sized form never exceeds the legacy
    'any call' size; at 128 < D <= 320 a run without Philox momenta (a replay tape, or a full cov_p,
    which takes the per-chain kernel) gets at least what the per-chain kernel needs; bad arguments
    size 0."""
    from hmc_amd import _lib as H
    monkeypatch.setattr(H, "_lib", None)
    L = H.lib()
    for D in (12, 100, 136, 300, 330):
        for iters in (1, 8, 32):
            for pm in (0, 1):
                ex = L.hmc_nuts_workspace_size_ex(D, 1000, 10, iters, pm)
                assert 0 < ex <= L.hmc_nuts_workspace_size(D, 1000, 10), (D, iters, pm)
    lock_philox = L.hmc_nuts_workspace_size_ex(200, 1000, 10, 8, 1)
    other = L.hmc_nuts_workspace_size_ex(200, 1000, 10, 8, 0)
    per_chain = L.hmc_nuts_workspace_size_ex(330, 1000, 10, 8, 0) * 200 // 330   # same layout, D-scaled
    assert other >= lock_philox and other >= per_chain * 0.9
    assert L.hmc_nuts_workspace_size_ex(100, 1000, 31, 8, 1) == 0          # d_max > 30
    assert L.hmc_nuts_workspace_size_ex(100, 1000, 30, 8, 1) > L.hmc_nuts_workspace_size_ex(100, 1000, 15, 8, 1)
    assert L.hmc_nuts_workspace_size_ex(100, 1000, 10, 0, 1) == 0          # iters_per_call < 1


def test_nuts_sized_entry_refuses_small_workspace(monkeypatch):
    """hmc_nuts_iters_ws checks the workspace size on the host before anything runs (advisor r04: a
    workspace sized for fewer Philox momentum iterations, or none, was a silent device overrun):
    EINVAL -> AssertionError, no GPU needed."""
    from hmc_amd import _lib as H
    monkeypatch.setattr(H, "_lib", None)
    L = H.lib()
    D, n, d_max = 100, 1000, 10
    T = H.Target(D, H.HMC_TARGET_DENSE, None, 1, 0.0)              # prec: any non-NULL pointer (not read)
    K = H.Kinetic(None, None, None, 0.1, None, None, None)
    st = H.State(1, 1)                                              # q, E_prev non-NULL (not read)
    S = H.Schedule(n, 0, 100, 0, 1, 101, 5, 20, 1, 33, H.HMC_RNG_PHILOX, H.HMC_MODE_FAST, d_max, 1, 0)
    small = L.hmc_nuts_workspace_size_ex(D, n, d_max, 8, 1)        # sized for 8 iterations per call
    with pytest.raises(AssertionError, match="needs"):
        H.check(L.hmc_nuts_iters_ws(T, K, S, None, st, 1, small, None), "x")     # a 32-iteration call
    none = L.hmc_nuts_workspace_size_ex(D, n, d_max, 32, 0)        # sized without Philox momenta
    with pytest.raises(AssertionError, match="needs"):
        H.check(L.hmc_nuts_iters_ws(T, K, S, None, st, 1, none, None), "x")


def test_every_scratch_entry_refuses_undersized_workspace(monkeypatch):
    """Every entry that takes device scratch refuses an undersized buffer on the host (HMC_EINVAL ->
    AssertionError) before a kernel could write past its end (verdict r05 item 4): the sized forms
    check the size they are given; the unsized forms check the size recorded for the buffer by a
    sized call or hmc_workspace_register.  Fake device pointers: nothing reaches the GPU."""
    from hmc_amd import _lib as H
    monkeypatch.setattr(H, "_lib", None)
    L = H.lib()
    K = H.Kinetic(None, None, None, 0.1, None, None, None)
    n = 1000
    S = H.Schedule(n, 0, 100, 0, 1, 101, 5, 20, 1, 11, H.HMC_RNG_PHILOX, H.HMC_MODE_FAST, 10, 1, 0)
    ORDER = 0x7000_0000                         # fake device pointers (never dereferenced here)
    for D, kind in ((100, H.HMC_TARGET_DENSE), (200, H.HMC_TARGET_DENSE), (3000, H.HMC_TARGET_DIAG)):
        T = H.Target(D, kind, None, 1 if kind == H.HMC_TARGET_DENSE else None, 0.0)
        need = L.hmc_random_workspace_size_ex(ctypes.byref(T), ctypes.byref(K), n)
        assert need > 0
        st = H.State(1, 1)
        st.order = ORDER
        with pytest.raises(AssertionError, match="needs"):
            H.check(L.hmc_random_iters_ws(T, K, S, None, st, need - 8, None), "x")
        with pytest.raises(AssertionError, match="needs"):
            H.check(L.hmc_chain_init_ws(T, K, S, None, 1, st, need - 8, None), "x")
        # unsized forms: a buffer recorded as too small is refused the same way
        assert L.hmc_workspace_register(ORDER, need - 8) == H.HMC_OK
        with pytest.raises(AssertionError, match="needs"):
            H.check(L.hmc_random_iters(T, K, S, None, st, None), "x")
        with pytest.raises(AssertionError, match="needs"):
            H.check(L.hmc_chain_init(T, K, S, None, 1, st, None), "x")
        assert L.hmc_workspace_register(ORDER, 0) == H.HMC_OK    # forget it
    # NUTS: the unsized entry refuses a workspace a sized call (or the caller) recorded as smaller
    D, d_max = 100, 10
    T = H.Target(D, H.HMC_TARGET_DENSE, None, 1, 0.0)
    st = H.State(1, 1)
    S32 = H.Schedule(n, 0, 100, 0, 1, 101, 5, 20, 1, 33, H.HMC_RNG_PHILOX, H.HMC_MODE_FAST, d_max, 1, 0)
    WS = 0x7100_0000
    small = L.hmc_nuts_workspace_size_ex(D, n, d_max, 8, 1)
    assert L.hmc_workspace_register(WS, small) == H.HMC_OK
    with pytest.raises(AssertionError, match="needs"):
        H.check(L.hmc_nuts_iters(T, K, S32, None, st, WS, None), "x")
    with pytest.raises(AssertionError, match="needs"):
        H.check(L.hmc_nuts_iters_ws(T, K, S32, None, st, WS, small, None), "x")
    assert L.hmc_workspace_register(WS, 0) == H.HMC_OK
    # a NULL kinetic block is refused, not dereferenced
    with pytest.raises(AssertionError):
        H.check(L.hmc_nuts_iters_ws(T, None, S32, None, st, WS, small, None), "x")
    with pytest.raises(AssertionError):
        H.check(L.hmc_workspace_register(None, 8), "x")
