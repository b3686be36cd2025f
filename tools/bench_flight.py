"""End-to-end latency of Flight.search against a fenix_amd.Server.

Not the headline metric (bench.py is); this measures what a fenix client sees:
descriptor pickling, gRPC DoExchange over loopback, io.index.call on the GPU,
the k-row gather and the result stream.  The server runs in this process; the
client runs in a child process that does not import torch (a torch import in
a client process alone costs ~10 ms per Flight round trip).  The
corpus is written through Flight.make_table as 1 000-row batches like the
reference's tests (test_flight.py:17-35); the first search stages the column
into HBM and is reported separately.

    python tools/bench_flight.py --n 100000 --d 128 --k 10 --metric l2
    python tools/bench_flight.py --n 1000000 --d 1536 --k 1000 --metric inner_product --dtype f16
"""

from __future__ import annotations

import argparse
import atexit
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402


def client(a) -> None:
    """Child process: no torch, only the Flight client."""
    import fenix_amd

    assert "torch" not in sys.modules
    f = fenix_amd.Flight(host="127.0.0.1", port=a.port)
    if a.read_all:  # the reference client's last step: FlightStreamReader.read_all()
        import pickle

        import pyarrow.flight as fl

        conn = f.conn

        def search(target, source, column, metric, maxval):
            cmd = {"coding": None, "source": source, "column": column, "metric": metric,
                   "select": None, "filter": pickle.dumps(None), "maxval": maxval,
                   "probes": None}
            table = pa.table({"target": pa.array(target)})
            w, r = conn.do_exchange(fl.FlightDescriptor.for_command(pickle.dumps(cmd)))
            with w:
                w.begin(table.schema)
                w.write_table(table)
                w.done_writing()
                return r.read_all()

        f = type("RefClient", (), {"search": staticmethod(search)})
    rs = np.random.RandomState(1)
    qs = rs.standard_normal((a.reps + 1, a.d)).astype(np.float16 if a.dtype == "f16" else np.float32)
    t0 = time.perf_counter()
    r = f.search(target=qs[0], source=a.source, column="vector", metric=a.metric,
                 maxval=a.k)
    first = time.perf_counter() - t0
    assert r.num_rows == a.k
    lat = []
    for i in range(a.reps):
        t0 = time.perf_counter()
        r = f.search(target=qs[i + 1], source=a.source, column="vector", metric=a.metric,
                     maxval=a.k)
        lat.append(time.perf_counter() - t0)
        assert r.num_rows == a.k
    print(json.dumps({"first_ms": first * 1e3, "lat_ms": [v * 1e3 for v in lat],
                      "torch_imported": "torch" in sys.modules}), flush=True)


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=100_000)
    p.add_argument("--d", type=int, default=128)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--metric", default="l2")
    p.add_argument("--dtype", default="f32", choices=["f32", "f16"])
    p.add_argument("--batch", type=int, default=1000)
    p.add_argument("--reps", type=int, default=30)
    p.add_argument("--clients", type=int, default=1, help="concurrent client processes")
    p.add_argument("--direct", action="store_true",
                   help="write the source file in-process (io.table.make) instead of "
                        "through Flight.make_table (large corpora)")
    p.add_argument("--root", default="", help="server root directory (default: a temp dir)")
    p.add_argument("--no-coalesce", action="store_true",
                   help="serve every request alone (FENIX_AMD_COALESCE=0)")
    p.add_argument("--canned", action="store_true",
                   help="the server answers every search with the first search's result "
                        "table (no io.index.call): the Flight + gRPC floor above the engine")
    p.add_argument("--read-all", action="store_true",
                   help="client: read the reply with FlightStreamReader.read_all() as the "
                        "reference's Flight.search does (flight.py:288)")
    p.add_argument("--client", action="store_true")
    p.add_argument("--port", type=int, default=0)
    p.add_argument("--source", default="bench/table", help="client: the table to search")
    a = p.parse_args()
    if a.client:
        return client(a)

    if a.no_coalesce:
        os.environ["FENIX_AMD_COALESCE"] = "0"
    import torch

    import fenix_amd
    from fenix_amd import coalesce
    from fenix_amd.engine import Engine

    eng = Engine.get(torch.device("cuda", 0))
    tdt = torch.float32 if a.dtype == "f32" else torch.float16
    vt = pa.list_(pa.float32() if a.dtype == "f32" else pa.float16(), a.d)
    schema = pa.schema({"id": pa.int64(), "vector": vt})

    def batches():
        dev = torch.empty((a.batch, a.d), dtype=tdt, device=eng.device)
        nb = (a.n + a.batch - 1) // a.batch
        for bi, s in enumerate(range(0, a.n, a.batch)):
            if nb >= 20 and bi % (nb // 10) == 0:
                print(f"ingest {bi}/{nb} batches", file=sys.stderr, flush=True)
            m = min(a.batch, a.n - s)
            eng.fill(dev[:m], seed=0, row_base=s)
            host = dev[:m].cpu().numpy()
            arr = pa.FixedSizeListArray.from_arrays(pa.array(host.ravel()), list_size=a.d)
            yield pa.record_batch([pa.array(np.arange(s, s + m, dtype=np.int64)), arr],
                                  names=["id", "vector"])

    root = tempfile.mkdtemp(prefix="fenix_bench_", dir=a.root or None)
    atexit.register(shutil.rmtree, root, True)  # (a 10M x 768 source is 30 GB of disk)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    server = fenix_amd.Server(root, host="127.0.0.1", port=port)
    writer = fenix_amd.Flight(host="127.0.0.1", port=port)
    t0 = time.perf_counter()
    reader = pa.RecordBatchReader.from_batches(schema, batches())
    if a.direct:
        from fenix_amd.io import table

        table.make(root, "bench/table", reader)
    else:
        writer.make_table("bench/table", reader)
    t_put = time.perf_counter() - t0
    if a.canned:
        from fenix_amd.io import index as _index

        real, memo = _index.call, {}

        def canned(*args, **kw):
            if "t" not in memo:
                memo["t"] = real(*args, **kw)
            return memo["t"]

        _index.call = canned
    cmd = [sys.executable, os.path.abspath(__file__), "--client", "--port", str(port),
           "--d", str(a.d), "--k", str(a.k), "--metric", a.metric, "--dtype", a.dtype,
           "--reps", str(a.reps)] + (["--read-all"] if a.read_all else [])
    t_all = time.perf_counter()
    procs = [subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for _ in range(a.clients)]
    outs = [p_.communicate(timeout=600) for p_ in procs]
    wall = time.perf_counter() - t_all
    server.shutdown()
    results = []
    for p_, (out, err) in zip(procs, outs):
        if p_.returncode != 0:
            print(err, file=sys.stderr)
            raise SystemExit(p_.returncode)
        results.append(json.loads(out.strip().splitlines()[-1]))
    res = results[0]
    lat = np.concatenate([np.array(r["lat_ms"]) for r in results])
    med = float(np.median(lat))
    print(json.dumps({
        "workload": f"{a.n}x{a.d} {a.dtype} {a.metric} k={a.k} via Flight.search "
                    "(loopback, torch-free client process)",
        "median_ms": med,
        "p90_ms": float(np.percentile(lat, 90)),
        "vectors_per_s": a.n / (med * 1e-3),
        "first_search_ms_incl_staging": res["first_ms"],
        "make_table_s": t_put,
        "ingest": "io.table.make in the server process" if a.direct else "Flight.make_table",
        "reps": a.reps,
        "client_imported_torch": res["torch_imported"],
        "clients": a.clients,
        "aggregate_searches_per_s": a.clients * a.reps / sum(
            np.sum(r["lat_ms"]) / 1e3 / a.clients for r in results) if a.clients > 1 else None,
        "wall_s_incl_client_start": wall,
        "canned_reply": a.canned,
        "client_read": "FlightStreamReader.read_all (the reference client)" if a.read_all
                       else "reader.to_reader().read_all() (fenix_amd.Flight.search)",
        "coalesce": coalesce.enabled(),
        "coalesced": coalesce.describe(coalesce.default()),
    }), flush=True)


if __name__ == "__main__":
    main()
