"""configs[4]'s per-GPU shard (6.25M x 1536 fp16, inner product, k = 1 000)
through the int8 filter image, query by query: candidate counts against the
buffer (an overflow falls back to the exact scan), time per search for the
image path and the exact scan, and whether the two return the same bits.

    python tools/k1000_sweep.py --queries 40 --opt i8_max_k=1024 --json out.json

Queries: ``--queries`` N(0,1) draws (seeds 1..), then as many "near" ones
(corpus row r + N(0,1)/2, r spread over the shard) and clustered-corpus runs
when ``--cluster`` is given.
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fenix_amd import _lib  # noqa: E402
from fenix_amd.engine import Engine, Shard  # noqa: E402


def timed(fn, reps):
    st = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    out = None
    for a, b in ev:
        a.record(st)
        out = fn()
        b.record(st)
    torch.cuda.synchronize()
    return out, float(np.median([a.elapsed_time(b) for a, b in ev]))


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=6_250_000)
    p.add_argument("--d", type=int, default=1536)
    p.add_argument("--k", type=int, default=1000)
    p.add_argument("--metric", default="inner_product")
    p.add_argument("--dtype", default="f16")
    p.add_argument("--queries", type=int, default=20)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--cluster", type=int, default=0)
    p.add_argument("--opt", action="append", default=[])
    p.add_argument("--json", default="")
    a = p.parse_args()
    for o in a.opt:
        name, value = o.split("=", 1)
        _lib.set_option(name, int(value))
    eng = Engine.get(torch.device("cuda", 0))
    tdt = torch.float16 if a.dtype == "f16" else torch.float32
    x = torch.empty((a.rows, a.d), dtype=tdt, device=eng.device)
    eng.fill(x, seed=0, cluster=a.cluster)
    shard = Shard(x, 0)
    m = _lib.METRICS[a.metric]
    qs = torch.empty((a.queries, a.d), dtype=torch.float32, device=eng.device)
    eng.fill(qs, seed=1)
    near_rows = np.linspace(0, a.rows - 1, a.queries).astype(np.int64)
    near = x[torch.from_numpy(near_rows).to(eng.device)].float() + 0.5 * qs
    recs = []
    for kind, Q in (("normal", qs), ("near", near)):
        for i in range(a.queries):
            q = Q[i : i + 1].contiguous()
            (ad, ar), t_img = timed(lambda: eng.search([shard], q, m, a.k), a.reps)
            st = eng.scan(shard, q, m, a.k)
            counts, cap = eng.filter_counts(shard, 1, m, a.k, st)
            with _lib.options(single_query_image=0):
                (ed, er), t_scan = timed(lambda: eng.search([shard], q, m, a.k), a.reps)
            same = bool(torch.equal(ar, er) and torch.equal(ad.view(torch.int32),
                                                           ed.view(torch.int32)))
            c = int(counts[0]) if counts is not None else -1
            recs.append({"kind": kind, "i": i, "count": c, "cap": cap, "overflow": c > cap,
                         "image_ms": t_img, "scan_ms": t_scan, "bit_identical": same})
            print(json.dumps(recs[-1]), flush=True)
    img = np.array([r["image_ms"] for r in recs])
    scan = np.array([r["scan_ms"] for r in recs])
    summary = {
        "workload": f"{a.rows}x{a.d} {a.dtype} {a.metric} k={a.k}, single queries"
                    + (f", clustered x{a.cluster}" if a.cluster else ""),
        "options": a.opt, "searches": len(recs),
        "overflowed": int(sum(r["overflow"] for r in recs)),
        "all_bit_identical": all(r["bit_identical"] for r in recs),
        "image_ms_median": float(np.median(img)), "image_ms_p90": float(np.percentile(img, 90)),
        "image_ms_max": float(img.max()), "scan_ms_median": float(np.median(scan)),
        "count_median": int(np.median([r["count"] for r in recs])),
        "count_max": int(max(r["count"] for r in recs)),
        "library_sha": _lib.library_sha(),
    }
    print(json.dumps(summary), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"summary": summary, "searches": recs}, f)
    if not summary["all_bit_identical"]:
        raise SystemExit("image path differs from the exact scan")


if __name__ == "__main__":
    main()
