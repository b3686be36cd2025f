"""End-to-end latency of Flight.search against a fenix_amd.Server (loopback).

Not the headline metric (bench.py is); this measures what a fenix client sees:
descriptor pickling, gRPC DoExchange, io.index.call on the GPU, the k-row
gather and the result stream.  Corpus written as an Arrow IPC stream of
1 000-row batches like the reference's tests (test_flight.py:17-35); the first
search stages the column into HBM and is reported separately.

    python tools/bench_flight.py --n 100000 --d 128 --k 10 --metric l2
    python tools/bench_flight.py --n 1000000 --d 1536 --k 1000 --metric inner_product --dtype f16
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=100_000)
    p.add_argument("--d", type=int, default=128)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--metric", default="l2")
    p.add_argument("--dtype", default="f32", choices=["f32", "f16"])
    p.add_argument("--batch", type=int, default=1000)
    p.add_argument("--reps", type=int, default=20)
    a = p.parse_args()

    import fenix_amd
    from fenix_amd.engine import Engine

    eng = Engine.get(torch.device("cuda", 0))
    tdt = torch.float32 if a.dtype == "f32" else torch.float16
    vt = pa.list_(pa.float32() if a.dtype == "f32" else pa.float16(), a.d)
    schema = pa.schema({"id": pa.int64(), "vector": vt})

    def batches():
        dev = torch.empty((a.batch, a.d), dtype=tdt, device=eng.device)
        for s in range(0, a.n, a.batch):
            m = min(a.batch, a.n - s)
            eng.fill(dev[:m], seed=0, row_base=s)
            host = dev[:m].cpu().numpy()
            arr = pa.FixedSizeListArray.from_arrays(pa.array(host.ravel()), list_size=a.d)
            yield pa.record_batch([pa.array(np.arange(s, s + m, dtype=np.int64)), arr],
                                  names=["id", "vector"])

    root = tempfile.mkdtemp(prefix="fenix_bench_")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    server = fenix_amd.Server(root, host="127.0.0.1", port=port)
    client = fenix_amd.Flight(host="127.0.0.1", port=port)
    t0 = time.perf_counter()
    client.make_table("bench/table", pa.RecordBatchReader.from_batches(schema, batches()))
    t_put = time.perf_counter() - t0
    qdev = torch.empty((a.reps + 1, a.d), dtype=torch.float32, device=eng.device)
    eng.fill(qdev, seed=1)
    qs = qdev.cpu().numpy().astype(np.float16 if a.dtype == "f16" else np.float32)
    t0 = time.perf_counter()
    r = client.search(target=qs[0], source="bench/table", column="vector", metric=a.metric,
                      maxval=a.k)
    t_first = time.perf_counter() - t0
    assert r.num_rows == a.k
    lat = []
    for i in range(a.reps):
        t0 = time.perf_counter()
        r = client.search(target=qs[i + 1], source="bench/table", column="vector",
                          metric=a.metric, maxval=a.k)
        lat.append(time.perf_counter() - t0)
        assert r.num_rows == a.k
    server.shutdown()
    med = float(np.median(lat))
    out = {
        "workload": f"{a.n}x{a.d} {a.dtype} {a.metric} k={a.k} via Flight.search (loopback)",
        "median_ms": med * 1e3,
        "p90_ms": float(np.percentile(lat, 90)) * 1e3,
        "vectors_per_s": a.n / med,
        "first_search_ms_incl_staging": t_first * 1e3,
        "make_table_s": t_put,
        "reps": a.reps,
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
