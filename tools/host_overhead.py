"""Host time to QUEUE one search (no synchronisation), per call path: what
delays the later devices of a single-process multi-GPU search
(engine._search_all queues device after device from one Python thread).

    python tools/host_overhead.py [--rows 1000000] [--d 768] [--k 100]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=1_000_000)
    p.add_argument("--d", type=int, default=768)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--reps", type=int, default=200)
    a = p.parse_args()
    import numpy as np
    import torch

    from fenix_amd import _lib, engine
    from fenix_amd.engine import Engine, Shard

    eng = Engine.get(torch.device("cuda", 0))
    x = torch.empty((a.rows, a.d), dtype=torch.float32, device=eng.device)
    eng.fill(x, seed=0)
    q = torch.from_numpy(np.random.RandomState(0).standard_normal((1, a.d)).astype(np.float32))
    qd = q.to(eng.device)
    sh = Shard(x, 0)
    m = _lib.METRICS["l2"]
    out = {}

    def timed(name, fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t0) * 1e6)
            torch.cuda.synchronize()
        out[name] = {"median_us": float(np.median(ts)), "p10_us": float(np.percentile(ts, 10))}
        print(name, json.dumps(out[name]), flush=True)

    with _lib.options(single_query_image=0):
        timed("engine_search_host_query", lambda: eng.search([sh], q, m, a.k))
        timed("engine_search_device_query", lambda: eng.search([sh], qd, m, a.k))
        od = torch.empty((1, a.k), dtype=torch.float32, device=eng.device)
        orow = torch.empty((1, a.k), dtype=torch.int64, device=eng.device)

        def raw():
            with eng.lock:
                eng.search_shard(sh, qd, m, a.k, None, od, orow)

        timed("search_shard", raw)
        timed("_search_all_one_shard", lambda: engine._search_all([sh], qd, m, a.k))
    print(json.dumps({"rows": a.rows, "d": a.d, "k": a.k, "host_us": out}), flush=True)


if __name__ == "__main__":
    main()
