"""ctypes binding of libhmc.so (the C ABI declared in include/hmc.h).

The product path has no CPU fallback: if the HIP library is missing or cannot
be loaded this module raises at import of the engine (`lib()`), loudly.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HMC_AMD_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libhmc.so"))

HMC_OK, HMC_EINVAL, HMC_EDMAX, HMC_EHIP, HMC_EINDEX, HMC_ENOTSUP = range(6)
HMC_TARGET_DIAG, HMC_TARGET_DENSE = 0, 1
HMC_RNG_REPLAY, HMC_RNG_PHILOX = 0, 1
HMC_MODE_EXACT, HMC_MODE_FAST = 0, 1
(CNT_ACCEPT, CNT_ACCEPT_WU, CNT_LEAPFROG, CNT_LEAPFROG_SQ, CNT_OOB_REJECT, CNT_UNSTABLE, CNT_DMAX,
 CNT_ENERGY_EVALS, CNT_HANDOFF_GIVEUP) = range(9)
NCOUNTERS = 9
COUNTER_SLOTS = 4096   # include/hmc.h HMC_COUNTER_SLOTS: counters buffer is [slots][NCOUNTERS]

c_dp = ctypes.c_void_p  # device pointers are passed as integers (torch data_ptr())


class Target(ctypes.Structure):
    _fields_ = [("D", ctypes.c_int32), ("kind", ctypes.c_int32), ("q0", c_dp), ("prec", c_dp),
                ("logdet_const", ctypes.c_double)]


class Kinetic(ctypes.Structure):
    _fields_ = [("minv", c_dp), ("p_scale", c_dp), ("dt_vec", c_dp), ("dt", ctypes.c_double),
                ("minv_full", c_dp), ("p_chol_t", c_dp), ("kick", c_dp)]


class Schedule(ctypes.Structure):
    _fields_ = [("n_chains", ctypes.c_int64), ("chain_offset", ctypes.c_int64), ("n_iter", ctypes.c_int32),
                ("warm_up", ctypes.c_int32), ("thin", ctypes.c_int32), ("L_chain", ctypes.c_int32),
                ("L_low", ctypes.c_int32), ("L_high", ctypes.c_int32), ("iter_begin", ctypes.c_int32),
                ("iter_end", ctypes.c_int32), ("rng_mode", ctypes.c_int32), ("fp_mode", ctypes.c_int32),
                ("d_max", ctypes.c_int32), ("on_dmax", ctypes.c_int32), ("seed", ctypes.c_uint64)]


class Replay(ctypes.Structure):
    _fields_ = [("p0", c_dp), ("p", c_dp), ("L", c_dp), ("lnu", c_dp), ("tape", c_dp),
                ("tape_stride", ctypes.c_int64)]


class State(ctypes.Structure):
    _fields_ = [("q", c_dp), ("E_prev", c_dp), ("q_chain", c_dp), ("E_chain", c_dp), ("dE_chain", c_dp),
                ("counters", c_dp), ("traj_q", c_dp), ("traj_len", c_dp), ("decision", c_dp),
                ("n_save", ctypes.c_int32), ("traj_stride", ctypes.c_int32),
                ("qc_rows", ctypes.c_int64), ("qc_row0", ctypes.c_int64), ("order", c_dp)]


# Exported symbols (tests check every one of these is present; keep in sync with include/hmc.h)
SYMBOLS = {
    "hmc_version": (ctypes.c_char_p, []),
    "hmc_last_error": (ctypes.c_char_p, []),
    "hmc_chain_init": (ctypes.c_int, [ctypes.POINTER(Target), ctypes.POINTER(Kinetic), ctypes.POINTER(Schedule),
                                      ctypes.POINTER(Replay), c_dp, ctypes.POINTER(State), c_dp]),
    "hmc_random_iters": (ctypes.c_int, [ctypes.POINTER(Target), ctypes.POINTER(Kinetic), ctypes.POINTER(Schedule),
                                        ctypes.POINTER(Replay), ctypes.POINTER(State), c_dp]),
    "hmc_chain_init_ws": (ctypes.c_int, [ctypes.POINTER(Target), ctypes.POINTER(Kinetic), ctypes.POINTER(Schedule),
                                         ctypes.POINTER(Replay), c_dp, ctypes.POINTER(State), ctypes.c_int64, c_dp]),
    "hmc_random_iters_ws": (ctypes.c_int, [ctypes.POINTER(Target), ctypes.POINTER(Kinetic),
                                           ctypes.POINTER(Schedule), ctypes.POINTER(Replay), ctypes.POINTER(State),
                                           ctypes.c_int64, c_dp]),
    "hmc_workspace_register": (ctypes.c_int, [c_dp, ctypes.c_int64]),
    "hmc_stream_work_size": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]),
    "hmc_stream_accumulate": (ctypes.c_int, [c_dp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                             ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_int64, ctypes.c_int32, c_dp, c_dp, c_dp, ctypes.c_int32, c_dp,
                                             c_dp, c_dp]),
    "hmc_random_workspace_size": (ctypes.c_int64, [ctypes.POINTER(Target), ctypes.c_int64]),
    "hmc_random_workspace_size_ex": (ctypes.c_int64, [ctypes.POINTER(Target), ctypes.POINTER(Kinetic),
                                                      ctypes.c_int64]),
    "hmc_nuts_workspace_size": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int64, ctypes.c_int32]),
    "hmc_nuts_workspace_size_ex": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                                    ctypes.c_int32]),
    "hmc_nuts_iters": (ctypes.c_int, [ctypes.POINTER(Target), ctypes.POINTER(Kinetic), ctypes.POINTER(Schedule),
                                      ctypes.POINTER(Replay), ctypes.POINTER(State), c_dp, c_dp]),
    "hmc_nuts_iters_ws": (ctypes.c_int, [ctypes.POINTER(Target), ctypes.POINTER(Kinetic), ctypes.POINTER(Schedule),
                                         ctypes.POINTER(Replay), ctypes.POINTER(State), c_dp, ctypes.c_int64, c_dp]),
    "hmc_leapfrog": (ctypes.c_int, [ctypes.POINTER(Target), ctypes.POINTER(Kinetic), ctypes.c_int64, c_dp, c_dp,
                                    c_dp, c_dp, ctypes.c_int32, c_dp]),
    "hmc_energy": (ctypes.c_int, [ctypes.POINTER(Target), ctypes.POINTER(Kinetic), ctypes.c_int64, c_dp, c_dp,
                                  c_dp, c_dp]),
    "hmc_rng_normals": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.c_int32, c_dp, c_dp]),
    "hmc_philox": (ctypes.c_int, [ctypes.c_uint32] * 6 + [ctypes.c_int64, c_dp, c_dp]),
    "hmc_split_moments": (ctypes.c_int, [c_dp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.c_int32, ctypes.c_int32, c_dp, c_dp, c_dp]),
    "hmc_rowsum_work_size": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32]),
    "hmc_rowsum": (ctypes.c_int, [c_dp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                  ctypes.c_int64, ctypes.c_int32, c_dp, c_dp, c_dp, c_dp]),
    "hmc_convergence_work_size": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]),
    "hmc_convergence_sums": (ctypes.c_int, [c_dp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                            ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, c_dp, c_dp, c_dp]),
    "hmc_half_sums": (ctypes.c_int, [c_dp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                     ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, c_dp, c_dp,
                                     c_dp]),
    "hmc_variogram_work_size": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]),
    "hmc_variogram": (ctypes.c_int, [c_dp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                     ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, c_dp, c_dp,
                                     c_dp]),
}

_lib = None


class HMCError(RuntimeError):
    pass


def lib():
    """Load libhmc.so once.  Raises (no fallback) when it is absent."""
    global _lib
    if _lib is None:
        path = os.environ.get("HMC_LIB_PATH", LIB_PATH)      # A/B builds of the same tree
        if not os.path.exists(path):
            raise RuntimeError(f"libhmc.so not found at {path}: build it with "
                               f"`python -c 'import __graft_entry__ as g; g.build()'` (make in csrc/)")
        L = ctypes.CDLL(path)
        for name, (res, args) in SYMBOLS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(status, what=""):
    """Map hmc_status to the exception type the reference raises for the same condition."""
    if status == HMC_OK:
        return
    msg = lib().hmc_last_error().decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if status in (HMC_EINVAL, HMC_EDMAX):
        raise AssertionError(text)       # reference validates with assert (samplers.py:331-348, :598)
    if status == HMC_EINDEX:
        raise IndexError(text)           # samplers.py:471 negative-index write (Q5)
    if status == HMC_ENOTSUP:
        raise NotImplementedError(text)
    raise HMCError(text)


def ptr(t):
    """Device pointer of a torch tensor (or None -> NULL)."""
    return None if t is None else t.data_ptr()
