"""Compare the final candidate sets of the two int8 batch kernels (option
img6 = 1 / 0) on the test's extreme-row corpus: rows appended by one only."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fenix_amd import _lib  # noqa: E402
from fenix_amd.engine import Engine, Shard  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.test_gpu_kernels import _extreme_rows  # noqa: E402

eng = Engine.get(torch.device("cuda", 0))
n, d, k, nq = 70_000, 136, 30, 65
xh = _extreme_rows(n, d, 49)
x = torch.from_numpy(xh).to(eng.device)
qh = O.fill_normal(nq, d, seed=60 + nq)
qh[3] = xh[17] * 2.0
q = torch.from_numpy(qh).to(eng.device)
m = _lib.METRICS[sys.argv[1] if len(sys.argv) > 1 else "l2"]
res = {}
for img6 in (1, 0):
    with _lib.options(img6=img6, filter_image=8):
        st = eng.scan(Shard(x, 0), q, m, k)
        counts, cap = eng.filter_counts(Shard(x, 0), nq, m, k, st)
        thr = torch.empty(nq, dtype=torch.int64, device=eng.device)
        cand = torch.empty((nq, cap), dtype=torch.int64, device=eng.device)
        cub = torch.empty((nq, cap), dtype=torch.int64, device=eng.device)
        _lib.check(_lib.load().fx_knn_filter_state(x.data_ptr(), 0, n, d, nq, m, k, 1,
                                                    st.ws.data_ptr(), st.ws.numel(),
                                                    thr.data_ptr(), cand.data_ptr(), cub.data_ptr(),
                                                    torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        res[img6] = (counts, thr.cpu().numpy(), cub.cpu().numpy().view(np.uint64))
c1, t1, u1 = res[1]
c0, t0, u0 = res[0]
print("thr equal", np.array_equal(t1, t0), "counts differ at", np.nonzero(c1 != c0)[0][:20])
for i in np.nonzero(c1 != c0)[0][:3]:
    r1 = set((u1[i, : min(c1[i], cap)] & np.uint64(0xffffffff)).tolist())
    r0 = set((u0[i, : min(c0[i], cap)] & np.uint64(0xffffffff)).tolist())
    extra1 = sorted(r1 - r0)[:5]
    extra0 = sorted(r0 - r1)[:5]
    print(f"q{i}: counts {c1[i]} vs {c0[i]}; only img6 {extra1}; only img3 {extra0}")
    for r in extra1:
        print("   row", r, "values max|x|", float(np.abs(xh[r]).max()), "finite", bool(np.isfinite(xh[r]).all()),
              "zero", not xh[r].any())
    allr = sorted(r1)
    print("   dup in img6:", len(allr) != int(min(c1[i], cap)))
