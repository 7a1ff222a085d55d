"""Dev timing of the one-read lag kernel (not a bench line), HIP events per call:
    python scripts/dev/lag_bench.py half N n D [reps]     hmc_half_sums over the second half of a window of
                                                          2n + 22 rows (c4: 131072 99 1000; no wrap, as
                                                          RandomEngine.run_streaming sizes c4's window)
    python scripts/dev/lag_bench.py halfwrap N n D [reps] the same over a half that wraps in a window of n + 22
    python scripts/dev/lag_bench.py conv N rows D [reps]  hmc_convergence_sums, every lag (tmax = n - 2)
                                                          of a stored (N, rows, D) window (c3: 262144 400 100;
                                                          headline: 1048576 100 100)
HMC_LIB_PATH selects an A/B build of the library."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "understanding-hmc_amd")]
from hmc_amd import _lib as H  # noqa: E402

mode = sys.argv[1]
N, n_or_rows, D = (int(v) for v in sys.argv[2:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
L = H.lib()
st = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device="cuda").manual_seed(1)
if mode in ("half", "halfwrap"):
    n = n_or_rows
    W = n + 22 if mode == "halfwrap" else 2 * n + 22
    x = torch.randn((N, W, D), dtype=torch.float64, device="cuda", generator=g)
    slot0 = W - 30 if mode == "halfwrap" else n + 1     # halfwrap: the half wraps after 30 samples
    T = max(1, n - 2)
    series_rows = n
    call = lambda work, out: L.hmc_half_sums(x.data_ptr(), N, x.stride(0), x.stride(1), D, W, slot0, n, T,  # noqa: E731
                                             H.ptr(work), H.ptr(out), st)
else:
    rows = n_or_rows
    x = torch.randn((N, rows, D), dtype=torch.float64, device="cuda", generator=g)
    n = rows // 2
    T = max(1, n - 2)
    series_rows = 2 * n
    call = lambda work, out: L.hmc_convergence_sums(x.data_ptr(), N, x.stride(0), x.stride(1), 0, n, D, T,  # noqa: E731
                                                    H.ptr(work), H.ptr(out), st)
for k in range(1, x.shape[1]):                         # AR(1)-ish rows (values only; the cost is data-blind)
    x[:, k].mul_(0.6).add_(x[:, k - 1], alpha=0.4)
work = torch.empty(L.hmc_convergence_work_size(N, D, T), dtype=torch.float64, device="cuda")
out = torch.empty((4 + T, D), dtype=torch.float64, device="cuda")
H.check(call(work, out), "lag pass")
torch.cuda.synchronize()
ts = []
for r in range(reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    H.check(call(work, out), "lag pass")
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ms = min(ts)
nbytes = N * series_rows * D * 8.0
fma = N * D * (series_rows // n) * sum(n - t for t in range(1, n))   # the reference loop's triangle
print(f"{mode} N={N} n={n} D={D} T={T}: ms {[round(t, 2) for t in ts]}  best {ms:.2f} ms  "
      f"{nbytes / ms / 1e6:.0f} GB/s of samples  {2 * fma / ms / 1e9:.1f} TFLOP/s (triangle FMAs)  "
      f"lib={os.environ.get('HMC_LIB_PATH', 'default')}", flush=True)
