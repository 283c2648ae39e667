"""HBM reference rates on this GPU: device copy (read + write), read-only
reduction, write-only fill.  Calibrates what the streaming passes can reach."""
import torch

n = 3_210_000_000 // 8  # 3.2 GB of u64, the bench's L1 key volume
a = torch.empty(n, dtype=torch.int64, device="cuda").random_(1 << 40)
b = torch.empty_like(a)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


ms = timed(lambda: b.copy_(a))
print(f"copy  {2 * a.nbytes / ms / 1e6:8.1f} GB/s  ({ms:.3f} ms for {a.nbytes / 1e9:.2f} GB read + write)")
ms = timed(lambda: a.sum())
print(f"read  {a.nbytes / ms / 1e6:8.1f} GB/s  ({ms:.3f} ms)")
ms = timed(lambda: b.fill_(7))
print(f"write {b.nbytes / ms / 1e6:8.1f} GB/s  ({ms:.3f} ms)")
