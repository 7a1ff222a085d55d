"""Per-phase breakdown of the NUTS wave step (debug build's s_memtime phase timers, not a bench line).
usage: HMC_LIB_PATH=understanding-hmc_amd/lib/libhmc_debug.so HMC_DEBUG_STAMPS=1 \
       python scripts/dev/nuts_phases.py [N] [S] [D] [rho] > out.json"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "understanding-hmc_amd")]
from hmc_amd.engine import NutsEngine  # noqa: E402
from hmc_amd.target import MVNTarget  # noqa: E402
from hmc_amd import _lib as H  # noqa: E402

a = sys.argv[1:] + ["65536", "16", "100", "0.95"][len(sys.argv) - 1:]
N, S, D, rho = int(a[0]), int(a[1]), int(a[2]), float(a[3])
assert os.environ.get("HMC_DEBUG_STAMPS") and "debug" in os.environ.get("HMC_LIB_PATH", "")
cov = (1 - rho) * np.eye(D) + rho
eng = NutsEngine(MVNTarget(np.zeros(D), cov), N, 3 * S, 0, 1, 10, 0.1, rng="philox", seed=0, fp_mode="fast",
                 store_chain=False, on_dmax="break")
q0 = torch.as_tensor(np.random.RandomState(0).standard_normal((N, D)) @ np.linalg.cholesky(cov).T).cuda()
eng.init(q0)
eng.run(1, 1 + S)                                  # warm-up launch
torch.cuda.synchronize()
c0 = eng.read_counters()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
eng.run(1 + S, 1 + 2 * S)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
c = eng.read_counters() - c0
L = H.lib()
L.hmc_debug_stamps.restype = ctypes.c_int64
L.hmc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
waves = min((N + 63) // 64, torch.cuda.get_device_properties(0).multi_processor_count) * 4
W = 16                                             # kStampWords (hmc_internal.hpp)
buf = np.zeros(waves * W, dtype=np.uint64)
got = L.hmc_debug_stamps(buf.ctypes.data, buf.size)
ph = buf[:got].reshape(-1, W).astype(np.float64)
tot = ph[:, :8].sum(axis=0)
sub = ph[:, 8:13].sum(axis=0)
end_steps = ph[:, 13].sum()
names = ["transitions", "kick+drift", "gradient (MFMA)", "kick+energies", "new point / saves",
         "loaded U-turn checks", "progressive sampling", "sub-tree end"]
sub_names = ["tree end (live point, row)", "write-back + drain + publish", "queue reservation",
             "poll + state loads", "momentum + tree start"]
steps = int(c[H.CNT_LEAPFROG_SQ])
out = dict(N=N, S=S, D=D, rho=rho, launch_ms=ms, leapfrogs=int(c[H.CNT_LEAPFROG]), wave_steps=steps,
           lane_utilisation=float(c[H.CNT_LEAPFROG]) / (16 * steps), lf_per_s=float(c[H.CNT_LEAPFROG]) / (ms / 1e3),
           waves=waves, phase_fraction={n: float(t / tot.sum()) for n, t in zip(names, tot)},
           phase_clk_per_step={n: float(t / max(steps, 1)) for n, t in zip(names, tot)},
           steps_with_tree_end=float(end_steps / max(steps, 1)),
           transition_clk_per_step={n: float(t / max(steps, 1)) for n, t in zip(sub_names, sub)},
           transition_clk_per_tree_end_step={n: float(t / max(end_steps, 1)) for n, t in zip(sub_names, sub)})
print(json.dumps(out, indent=1))
