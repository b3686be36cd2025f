"""Candidate counts of a batched / filter-image search (fx_knn_filter_counts):
how many (row, query) pairs the int8 bounds keep per query, against the
buffer's capacity (count > cap: the query overflowed).
    python tools/filter_counts.py [--rows N] [--d D] [--nq Q] [--k K] [--metric M]
                                  [--cluster C] [--query normal|near]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fenix_amd import _lib  # noqa: E402
from fenix_amd.engine import Engine, Shard  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--rows", type=int, default=10_000_000)
p.add_argument("--d", type=int, default=768)
p.add_argument("--nq", type=int, default=256)
p.add_argument("--k", type=int, default=100)
p.add_argument("--metric", default="cosine")
p.add_argument("--cluster", type=int, default=0)
p.add_argument("--query", default="normal")
p.add_argument("--opt", action="append", default=[])
a = p.parse_args()
for o in a.opt:
    name, value = o.split("=", 1)
    _lib.set_option(name, int(value))
eng = Engine.get(torch.device("cuda", 0))
x = torch.empty((a.rows, a.d), dtype=torch.float32, device=eng.device)
eng.fill(x, seed=0, cluster=a.cluster)
q = torch.empty((a.nq, a.d), dtype=torch.float32, device=eng.device)
eng.fill(q, seed=1)
if a.query == "near":
    q = x[a.rows // 3 : a.rows // 3 + 1] + 0.5 * q
m = _lib.METRICS[a.metric]
shard = Shard(x, 0)
st = eng.scan(shard, q, m, a.k)
counts, cap = eng.filter_counts(shard, a.nq, m, a.k, st)
c = counts.astype(np.int64)
print(json.dumps({"args": vars(a), "cap": cap, "overflowed": int((c > cap).sum()),
                  "count_p50": int(np.median(c)), "count_p90": int(np.percentile(c, 90)),
                  "count_max": int(c.max()), "counts": c.tolist()}))
