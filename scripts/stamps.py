"""Diagnostic: per-wave s_memtime phase timers of hmc_random_iters (HMC_DEBUG_STAMPS path)."""
import ctypes, os, sys
os.environ["HMC_DEBUG_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "understanding-hmc_amd"))
import numpy as np, torch
from hmc_amd.engine import RandomEngine
from hmc_amd.target import MVNTarget
from hmc_amd import _lib as H
L = H.lib()
L.hmc_debug_stamps.restype = ctypes.c_int64
L.hmc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
N, D = int(os.environ.get("N", 131072)), int(os.environ.get("DIM", 100))
eng = RandomEngine(MVNTarget(np.zeros(D), np.eye(D)), N, 40, 11, 1, 5, 20, 0.1, rng="philox", fp_mode="fast")
eng.init(torch.randn(N, D, dtype=torch.float64, device="cuda"))
eng.run(1, 11); torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); eng.run(11, 21); e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
buf = np.zeros(N * 8, dtype=np.uint64)
n = L.hmc_debug_stamps(buf.ctypes.data, buf.size)
w = buf[:n].reshape(-1, 8).astype(np.float64)
ph = w[:, :6].sum(0) / w.shape[0] / 10
life = w[:, 7] - w[:, 6]
t0 = w[:, 6].min(); span = w[:, 7].max() - t0
print("K=%s N=%d waves=%d kernel %.3f ms  stamp-span %.0f ticks -> %.3f GHz tick rate" % (
    os.environ.get("HMC_FORCE_K", "auto"), N, w.shape[0], ms, span, span / (ms * 1e6)))
print("  wave lifetime: mean %.0f ticks (%.1f%% of span); mean resident waves %.1f (per SIMD %.2f)" % (
    life.mean(), 100 * life.mean() / span, life.sum() / span, life.sum() / span / 1024))
names = ["momentum", "E0", "rowbook+L/u", "leapfrog", "E1", "MH+stores"]
for nm, x in zip(names, ph):
    print("  %-12s %9.0f ticks/wave-iter (%.1f%%)" % (nm, x, 100 * x / ph.sum()))
print("  unaccounted per wave (prologue/epilogue): %.0f ticks" % (life.mean() - w[:, :6].sum(1).mean()))
# ---- placement / concurrency (slot 5 high word = HW_ID, bits 16..31 = XCC_ID)
hw = (buf[:n].reshape(-1, 8)[:, 5] >> np.uint64(32)).astype(np.int64)
xcc = ((buf[:n].reshape(-1, 8)[:, 5] >> np.uint64(16)) & np.uint64(0xffff)).astype(np.int64)
simd = (hw >> 4) & 3; cu = (hw >> 8) & 15; sh = (hw >> 12) & 1; se = (hw >> 13) & 7; slot = hw & 15
key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
st, en = w[:, 6], w[:, 7]
print("  distinct SIMDs used:", len(np.unique(key)), " distinct XCC ids:", np.unique(xcc)[:10], " wave slots max:", slot.max())
conc = []
for k in np.unique(key)[:64]:
    m = key == k
    ev = np.concatenate([np.stack([st[m], np.ones(m.sum())], 1), np.stack([en[m], -np.ones(m.sum())], 1)])
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    c = np.cumsum(ev[:, 1])
    dur = np.diff(ev[:, 0])
    conc.append((c[:-1] * dur).sum() / max(dur.sum(), 1))
    if len(conc) == 1:
        print("  SIMD0: waves %d, max concurrent %d, busy span %.0f ticks" % (m.sum(), c.max(), ev[-1, 0] - ev[0, 0]))
print("  mean concurrent waves per SIMD (64 SIMDs sampled): %.2f" % np.mean(conc))
