"""Determinism check of the int8 filter kernels: the same search repeated,
per-query candidate counts compared across repetitions (a count that moves
means a kernel read data that had not landed).  Prints one line per case.

    python tools/race_check.py [--reps 30] [--nq 1,2,16,64,65,256] [--img6 0,1,2]
    FENIX_AMD_LIB=fenix_amd/lib/libfenix_knn_pe0.so python tools/race_check.py ...
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fenix_amd import _lib  # noqa: E402
from fenix_amd.engine import Engine, Shard, device_mask  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.test_gpu_kernels import _extreme_rows  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--reps", type=int, default=30)
p.add_argument("--nq", default="1,2,16,64,65,256", help="batch sizes (1-64: the q64i build)")
p.add_argument("--img6", default="0,1,2", help="option img6 values")
p.add_argument("--d", default="136,768")
p.add_argument("--img8", default="1", help="option img8 values (0: off, 1: filter_img8_kernel)")
p.add_argument("--metric", type=int, default=0, help="0 L2, 1 inner product, 2 cosine")
p.add_argument("--n", type=int, default=70_000,
               help="rows (600000 and up: a 3-phase plan, every int8 phase in the batched kernels)")
p.add_argument("--fp16", action="store_true",
               help="the fp16 filter kernels instead: fp16 image (k = 30) and no image (k = 300)")
a = p.parse_args()
eng = Engine.get(torch.device("cuda", 0))
k = 30
if a.fp16:
    for n, d in ((70_000, 136), (70_000, 768)):
        xh = _extreme_rows(n, d, 49)
        x = torch.from_numpy(xh).to(eng.device)
        for nq in (65, 256):
            q = torch.from_numpy(O.fill_normal(nq, d, seed=60 + nq)).to(eng.device)
            for name, opts, kk in (("fp16 image", {"filter_image": 16}, 30),
                                   ("no image", {"filter_image": 0}, 300)):
                eng.clear_images()
                with _lib.options(**opts):
                    ref, moved = None, 0
                    for _ in range(a.reps):
                        st = eng.scan(Shard(x, 0), q, 0, kk)
                        c, _cap = eng.filter_counts(Shard(x, 0), nq, 0, kk, st)
                        if c is None:
                            break
                        if ref is None:
                            ref = c
                        elif not np.array_equal(c, ref):
                            moved += 1
                    print(f"d {d} nq {nq} {name} k {kk}: "
                          + ("no filter" if ref is None else
                             f"{moved} of {a.reps - 1} repetitions moved"), flush=True)
    sys.exit(0)
for n, d in [(a.n, int(v)) for v in a.d.split(",")]:
    xh = _extreme_rows(n, d, 49)
    x = torch.from_numpy(xh).to(eng.device)
    eng.clear_images()
    mask = device_mask(np.random.RandomState(4).rand(n) < 0.8, eng.device)
    for nq in [int(v) for v in a.nq.split(",")]:
        q = torch.from_numpy(O.fill_normal(nq, d, seed=60 + nq)).to(eng.device)
        for msk in (None, mask):
            first = None
            for img6, img8 in [(int(v), int(w)) for v in a.img6.split(",") for w in a.img8.split(",")]:
                with _lib.options(img6=img6, img8=img8, filter_image=8, batch_min_queries=1):
                    ref = None
                    moved = 0
                    for _ in range(a.reps):
                        st = eng.scan(Shard(x, 0), q, a.metric, k, msk)
                        c, _cap = eng.filter_counts(Shard(x, 0), nq, a.metric, k, st)
                        if ref is None:
                            ref = c
                        elif not np.array_equal(c, ref):
                            moved += 1
                            diff = np.nonzero(c != ref)[0]
                            print(f"   d {d} nq {nq} mask {msk is not None} img6 {img6} img8 {img8}: "
                                  f"queries {diff[:20].tolist()} {(c[diff] - ref[diff])[:20].tolist()}",
                                  flush=True)
                    same = None
                    if first is None:
                        first = ref
                    else:
                        same = bool(np.array_equal(ref, first))
                    print(f"d {d} nq {nq} mask {msk is not None} img6 {img6} img8 {img8}: {moved} of "
                          f"{a.reps - 1} repetitions moved"
                          + ("" if same is None else f"; counts equal the first variant's: {same}"),
                          flush=True)
