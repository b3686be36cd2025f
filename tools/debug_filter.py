"""Debug a filter-image search against the exact scan: which true top-k rows
are missing from the final candidates, with their bounds.
    python tools/debug_filter.py [--metric l2] [--n 20000] [--d 64] [--nq 16] [--k 25] [--extreme]"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fenix_amd import _lib  # noqa: E402
from fenix_amd.engine import Engine, Shard  # noqa: E402
from oracle import oracle as O  # noqa: E402


def key_float(k):
    k = np.asarray(k, dtype=np.uint32)
    bits = np.where(k & 0x80000000, k & 0x7fffffff, ~k)
    return bits.astype(np.uint32).view(np.float32)


p = argparse.ArgumentParser()
p.add_argument("--metric", default="l2")
p.add_argument("--n", type=int, default=20000)
p.add_argument("--d", type=int, default=64)
p.add_argument("--nq", type=int, default=16)
p.add_argument("--k", type=int, default=25)
p.add_argument("--extreme", action="store_true")
a = p.parse_args()
eng = Engine.get(torch.device("cuda", 0))
xh = O.fill_normal(a.n, a.d, 31)
qh = O.fill_normal(a.nq, a.d, seed=32)
if a.extreme:  # tests/test_gpu_kernels.py::test_batched_filter_extreme_rows_and_queries
    rs = np.random.RandomState(5)
    big = rs.choice(a.n, 40, replace=False)
    xh[big[:10]] *= 1e5
    xh[big[10:20]] *= 1e-7
    xh[big[20:25], 3] = np.inf
    xh[big[25:30], 7] = np.nan
    xh[big[30:35]] = 0.0
    xh[big[35:40]] *= 3e4
    qh[0] *= 2.0 ** 60
    qh[1] *= 2.0 ** -60
    qh[2] = xh[big[0]]
    qh[3] = xh[big[12]]
    qh[4] = 0.0
    print("big rows", big.tolist())
x = torch.from_numpy(xh).to(eng.device)
q = torch.from_numpy(qh).to(eng.device)
m = _lib.METRICS[a.metric]
shard = Shard(x, 0)
st = eng.scan(shard, q, m, a.k)
counts, cap = eng.filter_counts(shard, a.nq, m, a.k, st)
thr = torch.empty(a.nq, dtype=torch.int64, device=eng.device)
cand = torch.empty((a.nq, cap), dtype=torch.int64, device=eng.device)
cub = torch.empty((a.nq, cap), dtype=torch.int64, device=eng.device)
_lib.check(_lib.load().fx_knn_filter_state(x.data_ptr(), 0, a.n, a.d, a.nq, m, a.k, 1,
                                            st.ws.data_ptr(), st.ws.numel(), thr.data_ptr(),
                                            cand.data_ptr(), cub.data_ptr(),
                                            torch.cuda.current_stream().cuda_stream))
od = torch.empty((a.nq, a.k), dtype=torch.float32, device=eng.device)
orow = torch.empty((a.nq, a.k), dtype=torch.int64, device=eng.device)
eng.reduce(shard, q, m, a.k, st, od, orow)
torch.cuda.synchronize()
with _lib.options(batched=0):
    sd, sr = eng.search([shard], q, m, a.k)
thr = thr.cpu().numpy().view(np.uint64)
cand = cand.cpu().numpy().view(np.uint64)
cub = cub.cpu().numpy().view(np.uint64)
print("cap", cap, "image", st.bits, "counts", counts.tolist())
fr, sr = orow.cpu().numpy(), sr.cpu().numpy()
for i in range(a.nq):
    c = min(int(counts[i]), cap)
    rows = (cand[i, :c] & np.uint64(0xffffffff)).astype(np.int64)
    ub_rows = (cub[i, :c] & np.uint64(0xffffffff)).astype(np.int64)
    lb = key_float(cand[i, :c] >> np.uint64(32))
    ub = key_float(cub[i, :c] >> np.uint64(32))
    same = np.array_equal(fr[i], sr[i])
    miss = [r for r in sr[i] if r not in set(rows.tolist())]
    print(f"q{i}: ok={same} count={counts[i]} thr={key_float(thr[i] >> np.uint64(32))} "
          f"rows_match_ub={np.array_equal(rows, ub_rows)} missing={len(miss)} dup={c - len(set(rows.tolist()))}")
    if not same:
        dist = O.distances(xh[sr[i]], qh[i:i+1], a.metric)[0]
        print("   true top rows", sr[i][:8], "dist", dist[:8])
        print("   got rows     ", fr[i][:8])
        uj = [np.nonzero(ub_rows == r)[0] for r in miss[:5]]
        for r, jj in zip(miss[:5], uj):
            print("   missing", r, "in ub list at", jj[:3], "ub", ub[jj[:3]] if len(jj) else None)
        j = np.nonzero(np.isin(rows, sr[i]))[0][:5]
        print("   present lb/ub", list(zip(rows[j], lb[j], ub[j])))
