"""Where io.index.call spends its time (server side of Flight.search), in-process.

    python tools/profile_call.py --n 1000000 --d 1536 --k 1000 --dtype f16
"""

from __future__ import annotations

import argparse
import cProfile
import os
import pstats
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402
import torch  # noqa: E402

from fenix_amd.engine import Engine  # noqa: E402
from fenix_amd.io import index, table  # noqa: E402


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1_000_000)
    p.add_argument("--d", type=int, default=1536)
    p.add_argument("--k", type=int, default=1000)
    p.add_argument("--dtype", default="f16")
    p.add_argument("--metric", default="inner_product")
    p.add_argument("--reps", type=int, default=20)
    a = p.parse_args()
    eng = Engine.get(torch.device("cuda", 0))
    tdt = torch.float16 if a.dtype == "f16" else torch.float32
    vt = pa.list_(pa.float16() if a.dtype == "f16" else pa.float32(), a.d)
    root = tempfile.mkdtemp(prefix="fenix_prof_")
    dev = torch.empty((100_000, a.d), dtype=tdt, device=eng.device)
    batches = []
    for s in range(0, a.n, 100_000):
        m = min(100_000, a.n - s)
        eng.fill(dev[:m], seed=0, row_base=s)
        host = dev[:m].cpu().numpy()
        arr = pa.FixedSizeListArray.from_arrays(pa.array(host.ravel()), list_size=a.d)
        for c in range(0, m, 1000):
            batches.append(pa.record_batch([pa.array(np.arange(s + c, s + c + min(1000, m - c),
                                                               dtype=np.int64)),
                                            arr.slice(c, min(1000, m - c))], names=["id", "vector"]))
    table.make(root, "p/t", pa.RecordBatchReader.from_batches(
        pa.schema({"id": pa.int64(), "vector": vt}), batches))
    q = np.random.RandomState(0).standard_normal(a.d).astype(np.float32)
    index.call(root, None, "p/t", "vector", target=q, metric=a.metric, maxval=a.k)  # stage
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        index.call(root, None, "p/t", "vector", target=q, metric=a.metric, maxval=a.k)
        ts.append((time.perf_counter() - t0) * 1e3)
    print("index.call ms: median %.3f min %.3f" % (np.median(ts), np.min(ts)), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.reps):
        index.call(root, None, "p/t", "vector", target=q, metric=a.metric, maxval=a.k)
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(30)


if __name__ == "__main__":
    main()
