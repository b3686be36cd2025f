"""Where io.index.call spends its time (server side of Flight.search), in-process.

    python tools/profile_call.py --n 1000000 --d 1536 --k 1000 --dtype f16
    # configs[4]'s serving shape on one GPU: 8 row shards of 500k x 1536 fp16
    python tools/profile_call.py --n 4000000 --shards 8 --batch 100000 --json out.json

Prints the median of ``--reps`` warm calls, a per-phase breakdown (each phase
wrapped with a wall clock; ``search_host`` ends with the result's D2H, which
waits for the GPU) and a cProfile listing.  ``--cpu-load`` runs the oracle's
16-thread OpenMP scan between calls, as tests/test_gpu_serving.py does, to
measure what that does to the next call.
"""

from __future__ import annotations

import argparse
import atexit
import collections
import cProfile
import json
import os
import pstats
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1_000_000)
    p.add_argument("--d", type=int, default=1536)
    p.add_argument("--k", type=int, default=1000)
    p.add_argument("--dtype", default="f16")
    p.add_argument("--metric", default="inner_product")
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--shards", type=int, default=1,
                   help="row shards on GPU 0 (FENIX_AMD_DEVICES=0,...,0)")
    p.add_argument("--batch", type=int, default=1000, help="rows per Arrow record batch")
    p.add_argument("--cpu-load", action="store_true",
                   help="also time calls that follow a 16-thread oracle scan")
    p.add_argument("--json", default="", help="write the timings here")
    a = p.parse_args()
    if a.shards > 1:
        os.environ["FENIX_AMD_DEVICES"] = ",".join(["0"] * a.shards)

    import numpy as np
    import pyarrow as pa
    import torch

    from fenix_amd.engine import Engine
    from fenix_amd.io import index, table

    eng = Engine.get(torch.device("cuda", 0))
    tdt = torch.float16 if a.dtype == "f16" else torch.float32
    vt = pa.list_(pa.float16() if a.dtype == "f16" else pa.float32(), a.d)
    root = tempfile.mkdtemp(prefix="fenix_prof_")
    atexit.register(shutil.rmtree, root, True)  # (a 10M x 768 source is 30 GB of disk)
    dev = torch.empty((100_000, a.d), dtype=tdt, device=eng.device)

    def batches():
        for s in range(0, a.n, 100_000):
            m = min(100_000, a.n - s)
            eng.fill(dev[:m], seed=0, row_base=s)
            host = dev[:m].cpu().numpy()
            arr = pa.FixedSizeListArray.from_arrays(pa.array(host.ravel()), list_size=a.d)
            for c in range(0, m, a.batch):
                w = min(a.batch, m - c)
                yield pa.record_batch([pa.array(np.arange(s + c, s + c + w, dtype=np.int64)),
                                       arr.slice(c, w)], names=["id", "vector"])

    table.make(root, "p/t", pa.RecordBatchReader.from_batches(
        pa.schema({"id": pa.int64(), "vector": vt}), batches()))
    del dev
    qs = np.random.RandomState(0).standard_normal((a.reps + 1, a.d)).astype(np.float32)
    t0 = time.perf_counter()
    index.call(root, None, "p/t", "vector", target=qs[0], metric=a.metric, maxval=a.k)  # stage
    first = (time.perf_counter() - t0) * 1e3
    print(f"first call (staging) {first:.1f} ms", flush=True)

    # phase clocks: wrap the functions io.index.call goes through
    phases = collections.defaultdict(list)

    # and a timeline of each call: (function, start, end) in us from the call's start
    events: list = []

    def clocked(mod, name, phase=True):
        fn = getattr(mod, name)

        def wrapper(*args, **kw):
            t = time.perf_counter()
            try:
                return fn(*args, **kw)
            finally:
                e = time.perf_counter()
                if phase:
                    phases[name].append((e - t) * 1e3)
                events.append((name, t, e))

        setattr(mod, name, wrapper)
        return fn

    for mod, name in ((index._resident, "sources"), (index._resident, "shards"),
                      (index, "_target_values"), (index._engine, "search_host"),
                      (index, "_take_columns"), (index, "_gather_vectors"),
                      (index, "_take_chunked")):
        clocked(mod, name)
    from fenix_amd import coalesce, engine

    for mod, name in ((engine, "_search_all"), (engine.Engine, "search"),
                      (engine.Engine, "search_shard"), (engine.Engine, "filter_image"),
                      (engine, "gather_rows"), (engine, "_to_host"), (engine, "check_rows"),
                      (coalesce.Coalescer, "search")):
        clocked(mod, name, phase=False)
    timeline = []

    def run(qi: int) -> float:
        events.clear()
        t = time.perf_counter()
        r = index.call(root, None, "p/t", "vector", target=qs[qi], metric=a.metric, maxval=a.k)
        e = time.perf_counter()
        ms = (e - t) * 1e3
        assert r.num_rows == a.k
        timeline[:] = [("index.call", t, e)] + sorted(events, key=lambda v: v[1])
        return ms

    ts = [run(1 + i) for i in range(a.reps)]
    t0 = timeline[0][1]
    print("timeline of the last call (us from its start: start, end, duration):")
    for name, s_, e_ in timeline:
        print(f"  {(s_ - t0) * 1e6:8.1f} {(e_ - t0) * 1e6:8.1f} {(e_ - s_) * 1e6:8.1f}  {name}")
    print("index.call ms: median %.3f min %.3f max %.3f" % (np.median(ts), min(ts), max(ts)),
          flush=True)
    breakdown = {k: float(np.median(v)) for k, v in phases.items()}
    print("phase medians (ms):", json.dumps(breakdown), flush=True)
    loaded = []
    if a.cpu_load:
        from oracle import oracle as O

        x = O.fill_normal_c(200_000, a.d, 5).astype(np.float16 if a.dtype == "f16" else np.float32)
        for i in range(5):
            O.knn(x, qs[i : i + 1].astype(np.float32), a.metric, a.k, threads=16)
            loaded.append(run(1 + i))
        print("after a 16-thread oracle scan, ms:", ["%.2f" % v for v in loaded], flush=True)

    pr = cProfile.Profile()
    pr.enable()
    for i in range(a.reps):
        run(1 + i)
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(35)
    pstats.Stats(pr).sort_stats("tottime").print_stats(40)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"workload": f"{a.n}x{a.d} {a.dtype} {a.metric} k={a.k}, "
                                   f"{a.shards} shard(s) on GPU 0, {a.batch}-row batches",
                       "first_call_ms": first, "call_ms": ts, "median_ms": float(np.median(ts)),
                       "phase_median_ms": breakdown, "after_cpu_load_ms": loaded}, f)


if __name__ == "__main__":
    main()
