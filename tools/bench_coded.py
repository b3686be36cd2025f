"""Coded-index kernels on one MI355X (not the headline metric; bench.py is).

* encode    fx_code_assign over the whole corpus (index.make's work,
            index.py:37-65): 2*n*nb*ks*d flops on MFMA + n*d*4 bytes;
* kmeans    one fx_kmeans_step of every codebook (coder.make's inner step,
            coder.py:118);
* probe     one probe search as io.index.call runs it (index.py:113-168):
            target -> codeword distances -> fx_code_probe -> fx_code_mask over
            the resident code column -> masked scan + merge, next to the exact
            full scan of the same corpus.

    python tools/bench_coded.py --n 10000000 --d 768 --nb 2 --ks 256 --probes 64
"""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from fenix_amd import _lib  # noqa: E402
from fenix_amd.engine import Engine, Shard  # noqa: E402


def timed(fn, iters):
    ts = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    v = sorted(a.elapsed_time(b) for a, b in ts)
    return v[len(v) // 2]


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--d", type=int, default=768)
    p.add_argument("--nb", type=int, default=2)
    p.add_argument("--ks", type=int, default=256)
    p.add_argument("--bs", type=int, default=25_600)
    p.add_argument("--probes", type=int, default=64)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--metric", default="l2")
    p.add_argument("--dtype", default="f32", choices=["f32", "f16"])
    p.add_argument("--iters", type=int, default=5)
    a = p.parse_args()
    m = _lib.METRICS[a.metric]
    eng = Engine.get(torch.device("cuda", 0))
    tdt = torch.float32 if a.dtype == "f32" else torch.float16
    x = torch.empty((a.n, a.d), dtype=tdt, device=eng.device)
    eng.fill(x, seed=0, cluster=1000)  # clustered rows: codes are informative
    g = torch.Generator().manual_seed(0)
    pick = torch.randperm(a.n, generator=g)[: a.nb * a.ks].sort().values.to(eng.device)
    cw = x.index_select(0, pick).to(torch.float32).reshape(a.nb, a.ks, a.d).contiguous()
    q = torch.empty((1, a.d), dtype=torch.float32, device=eng.device)
    eng.fill(q, seed=1)
    out = {"workload": f"{a.n}x{a.d} {a.dtype} {a.metric}, {a.nb} codebooks x {a.ks}",
           "n": a.n, "d": a.d, "nb": a.nb, "ks": a.ks}

    # encode
    eng.code_assign(x, cw, m)
    ms = timed(lambda: eng.code_assign(x, cw, m), a.iters)
    flops = 2.0 * a.n * a.nb * a.ks * a.d
    out["encode_ms"] = ms
    out["encode_tflops"] = flops / ms / 1e9
    out["encode_gbs"] = a.n * a.d * x.element_size() / ms / 1e6
    _, codes, _ = eng.code_assign(x, cw, m)

    # k-means step
    bs = min(a.bs, a.n // a.nb)
    sample = x[: a.nb * bs].reshape(a.nb, bs, a.d)
    work = cw.clone()
    eng.kmeans_step(sample, work, m)
    out["kmeans_bs"] = bs
    out["kmeans_step_ms"] = timed(lambda: eng.kmeans_step(sample, work, m), a.iters)

    # probe search vs exact full scan
    shard = Shard(x, 0)
    total = a.ks**a.nb

    def probe_search(row_list=True):
        dq = eng.distances(Shard(cw.reshape(a.nb * a.ks, a.d), 0), q, m)
        _, _, sel = eng.code_probe(dq.reshape(1, a.nb, a.ks), a.probes)
        mk, cnt = eng.code_mask(codes, sel[0], total)
        c = int(cnt.item())  # index.call reads the count (maxval branch, index.py:165)
        return eng.search([shard], q, m, a.k, [mk], [c] if row_list else None), c

    (_, _), kept = probe_search()
    out["probes"] = a.probes
    out["probe_rows_kept"] = kept
    out["probe_search_ms"] = timed(probe_search, a.iters)
    out["probe_search_masked_scan_ms"] = timed(lambda: probe_search(False), a.iters)
    dq = eng.distances(Shard(cw.reshape(a.nb * a.ks, a.d), 0), q, m)
    out["probe_select_ms"] = timed(lambda: eng.code_probe(dq.reshape(1, a.nb, a.ks), a.probes),
                                   a.iters)
    eng.search([shard], q, m, a.k)
    out["full_search_ms"] = timed(lambda: eng.search([shard], q, m, a.k), a.iters)
    kept = out["probe_rows_kept"]
    out["probe_scan_gbs_effective"] = kept * a.d * x.element_size() / out["probe_search_ms"] / 1e6
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
