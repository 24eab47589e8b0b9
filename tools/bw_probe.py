"""HBM bandwidth calibration on the box: torch's own streaming kernels over 2^26 int64 (512 MiB)."""
import torch

n = 1 << 26
x = torch.ones(n, dtype=torch.int64, device="cuda")
y = torch.empty_like(x)
s = torch.cuda.current_stream()


def t(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / reps / 1e3


nb = n * 8
print(f"read (sum)   {nb / t(lambda: x.sum()) / 1e12:.2f} TB/s")
print(f"write (fill) {nb / t(lambda: y.fill_(3)) / 1e12:.2f} TB/s")
print(f"copy         {2 * nb / t(lambda: y.copy_(x)) / 1e12:.2f} TB/s (read + write)")
