"""Random row fetch rate: torch index_select of R random 3 KB rows from a
corpus of N rows (768 f32), N = 100K .. 10M; shows whether the rescoring
kernels' ~250 rows/us is a property of random row access over a large
allocation (address translation) rather than of the kernels."""
import torch

d = 768
for n in (100_000, 1_000_000, 10_000_000):
    x = torch.empty((n, d), dtype=torch.float32, device="cuda")
    x.normal_()
    for r in (25_600, 100_000):
        idx = torch.randint(0, n, (r,), device="cuda")
        y = x.index_select(0, idx)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            y = x.index_select(0, idx)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / 10
        print(f"n={n:>10} rows={r:>7}: {us:8.1f} us  {r / us:7.1f} rows/us  {r * d * 4 / us / 1e3:6.2f} TB/s",
              flush=True)
    del x
    torch.cuda.empty_cache()
