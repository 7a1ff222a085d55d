"""Calibration for FETCH_SIZE / WRITE_SIZE on this box: kernels with known byte counts.
fill: writes 1 GiB; copy: reads 1 GiB + writes 1 GiB (torch elementwise kernels, 16 B/lane)."""
import torch
n = 1 << 27  # doubles = 1 GiB
a = torch.empty(n, dtype=torch.float64, device="cuda")
b = torch.empty_like(a)
for _ in range(3):
    a.fill_(1.0)
    b.copy_(a)
torch.cuda.synchronize()
print("calib done")
