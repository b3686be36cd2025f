"""Time the batched filter search under FX_FILTER_DIAG variants (profiling aid,
not part of the product): 0 full, 1 no appends, 2 no epilogue, 4 no MFMA.

    python tools/filter_diag.py [--n 10000000] [--d 768] [--nq 256] [--metric cosine]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fenix_amd import _lib  # noqa: E402
from fenix_amd.engine import Engine, Shard  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--d", type=int, default=768)
    p.add_argument("--nq", type=int, default=256)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--metric", default="cosine")
    p.add_argument("--iters", type=int, default=3)
    p.add_argument("--diags", default="0,1,2,3,4,6,7")
    p.add_argument("--dtype", default="f32", choices=["f32", "f16"])
    p.add_argument("--envs", default="", help="';'-separated NAME=VALUE settings to A/B, e.g. FX_FILTER2=0;FX_FILTER2=1")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    eng = Engine.get(dev)
    x = torch.empty((a.n, a.d), dtype=torch.float16 if a.dtype == "f16" else torch.float32,
                    device=dev)
    eng.fill(x, seed=0)
    q = torch.empty((a.nq, a.d), dtype=torch.float32, device=dev)
    eng.fill(q, seed=1)
    shard = Shard(x, 0)
    metric = _lib.METRICS[a.metric]
    settings = [e for e in a.envs.split(";") if e] or [""]
    runs = [(dg, e) for _ in range(2) for e in settings for dg in [int(v) for v in a.diags.split(",")]]
    for dg, env in runs:
        if env:
            k, v = env.split("=", 1)
            os.environ[k] = v
        os.environ["FX_FILTER_DIAG"] = str(dg)
        eng.scan(shard, q, metric, a.k)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.scan(shard, q, metric, a.k)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(json.dumps({"diag": dg, "env": env, "lib": os.path.basename(_lib.LIB_PATH),
                          "ms": float(np.median(ts))}), flush=True)
    os.environ.pop("FX_FILTER_DIAG")


if __name__ == "__main__":
    main()
