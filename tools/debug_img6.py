"""Repeat one int8 filter search with the resident-slice kernel (img6=2) and
compare the final candidate sets between repetitions: rows appended in one
run only, with their image position (tile, wave row block, lane) and the
phase threshold.  Also the streamed-tile kernel (img6=0) once as reference."""
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
n, d, k, nq = 70_000, int(sys.argv[1]) if len(sys.argv) > 1 else 768, 30, 65
xh = _extreme_rows(n, d, 49)
x = torch.from_numpy(xh).to(eng.device)
qh = O.fill_normal(nq, d, seed=60 + nq)
q = torch.from_numpy(qh).to(eng.device)
m = 0
L = _lib.load()
perm_a = _lib.image8_perm(n)


def run(img6):
    with _lib.options(img6=img6, filter_image=8):
        st = eng.scan(Shard(x, 0), q, m, k)
        counts, cap = eng.filter_counts(Shard(x, 0), nq, m, k, st)
        thr = torch.empty(nq, dtype=torch.int64, device=eng.device)
        cand = torch.empty((nq, cap), dtype=torch.int64, device=eng.device)
        cub = torch.empty((nq, cap), dtype=torch.int64, device=eng.device)
        _lib.check(L.fx_knn_filter_state(x.data_ptr(), 0, n, d, nq, m, k, 1, st.ws.data_ptr(),
                                         st.ws.numel(), thr.data_ptr(), cand.data_ptr(),
                                         cub.data_ptr(), torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        return counts, thr.cpu().numpy(), cub.cpu().numpy().view(np.uint64), cap


def rows_of(res, i):
    c, _, cand, cap = res
    return cand[i, : min(c[i], cap)]


ref = run(0)
runs = [run(2) for _ in range(6)]
pinv = {}
for r in range(len(runs)):
    c = runs[r][0]
    dq = np.nonzero(c != ref[0])[0]
    print(f"run {r}: thr equal {np.array_equal(runs[r][1], ref[1])}; queries differing from img3 "
          f"{dq.tolist()[:20]} by {(c[dq].astype(np.int64) - ref[0][dq])[:5].tolist()}")
    for i in dq[:2]:
        a = {int(e & 0xffffffff): int(e >> 32) for e in rows_of(runs[r], i)}
        b = {int(e & 0xffffffff): int(e >> 32) for e in rows_of(ref, i)}
        only6 = sorted(set(a) - set(b))
        only3 = sorted(set(b) - set(a))
        dif = [(rw, a[rw], b[rw]) for rw in set(a) & set(b) if a[rw] != b[rw]][:5]
        print(f"   q{i}: only img6 {only6[:6]} only img3 {only3[:6]} same row, other key {dif}")
        lst = rows_of(runs[r], i)
        rws = (lst & np.uint64(0xffffffff)).astype(np.int64)
        u, cnt = np.unique(rws, return_counts=True)
        dup = u[cnt > 1]
        for rw in dup[:3]:
            slots = np.nonzero(rws == rw)[0]
            print(f"      duplicate row {rw} at slots {slots.tolist()} of {len(lst)}, keys "
                  f"{[hex(int(lst[s_] >> 32)) for s_ in slots]}; image row "
                  f"{int((rw * pow(int(perm_a), -1, n)) % n)}")
        ub = runs[r][2]
        for rw in (only6 + only3)[:4]:
            # image position of corpus row rw: i with (a i) mod n == rw
            pos = None
            if perm_a:
                pos = int((rw * pow(int(perm_a), -1, n)) % n)
            print(f"      row {rw}: image row {pos} (tile {pos // 256 if pos is not None else None}, "
                  f"block {(pos % 256) // 32 if pos is not None else None}, lane {pos % 32 if pos is not None else None}), "
                  f"max|x| {float(np.abs(xh[rw]).max()):.3g} zero {not xh[rw].any()} "
                  f"finite {bool(np.isfinite(xh[rw]).all())}")
