"""BASELINE configs[4]'s serving combination as one test, at a size one GPU
can stage: Flight.make_table of a 1536-d float16 source (8 x 500 000 rows),
then Flight.search (flight.py:242-288) -> Server.do_exchange (flight.py:62-77)
-> io.index.call -> the 8-shard search (FENIX_AMD_DEVICES=0,0,0,0,0,0,0,0:
eight row shards on the one GPU, exactly the 8-GPU deployment's split and
merge) -> inner product, k = 1 000 -> the ~3 MB reply with every column.
Row ids are checked against the float64 oracle, the gathered vectors against
the source rows, the halffloat distances at fp16 resolution.

The latency is timed the way a client sees it: a torch-free client process
(tools/bench_flight.py --client) over loopback gRPC, 20 warm searches, with a
bound on the median.  The checks above run in this process, which also hosts
the server; a search timed from here measured 28-29 ms in round 4 against
5.3 ms from a separate client (profiles/r05_cfg4_serving_test.json): the
in-process client shares the server's interpreter and GIL, and this process
imports torch, which a client never does."""

from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pyarrow as pa
import pytest
import torch

import fenix_amd
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SHARDS, PER_SHARD, D, K = 8, 500_000, 1536, 1000
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# median of 20 warm searches from a separate client process (5.3 ms before the
# one-sync vector gather, profiles/r05_cfg4_serving_test.json; 3.74 ms after,
# profiles/r05_cfg4_serving_test2.json; 4.70 ms on another box,
# profiles/r06_cfg4_serving_test.json).  A guard against a gross regression
# (round 4's in-process client measured 28 ms), set well above box-to-box
# variation so that timing noise alone cannot fail this correctness test
# (ADVICE r5); the median itself is recorded in gpurun_out/cfg4_serving_test.json.
MEDIAN_MS_BOUND = 8.0
# positions (of 3 queries x 1 000) whose id differs from the float64 oracle at
# a near-tie (tests/parity.py's rule): float32 accumulation cannot order rows
# whose 1536-d fp16 inner products differ by < 2e-6 relative.  Measured: 2
# (profiles/r05_cfg4_serving_test2.json).
NEAR_TIE_CAP = 6
VECTOR = pa.list_(pa.float16(), D)
SCHEMA = pa.schema({"id": pa.int64(), "vector": VECTOR})


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _reader(x16: np.ndarray, batch: int = 100_000) -> pa.RecordBatchReader:
    def gen():
        for s in range(0, x16.shape[0], batch):
            part = x16[s : s + batch]
            a = pa.FixedSizeListArray.from_arrays(pa.array(part.ravel()), list_size=D)
            i = pa.array(np.arange(s, s + len(part), dtype=np.int64))
            yield pa.record_batch([i, a], names=["id", "vector"])

    return pa.RecordBatchReader.from_batches(SCHEMA, gen())


def _check_ids(ids, orow, od, x16, qh):
    """Row ids equal the float64 oracle's except at near-ties (tests/parity.py's
    rule: float64 inner products closer than 2e-6 of |q| max|x|, which the
    float32 accumulation cannot order); returns how many positions used one."""
    if np.array_equal(ids, orow):
        return 0
    diff = np.nonzero(ids != orow)[0]
    xn = float(np.sqrt((x16[ids].astype(np.float64) ** 2).sum(axis=1)).max())
    near = 2e-6 * float(np.sqrt((qh.astype(np.float64) ** 2).sum())) * xn
    d_gpu_rows = O.distances(x16[ids[diff]], qh, "inner_product")[0]
    assert np.all(np.abs(d_gpu_rows - od[diff]) <= near), (diff, d_gpu_rows, od[diff], near)
    return len(diff)


def test_configs4_flight_8_shards_f16_ip_k1000(tmp_path, monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fenix_amd import engine

    monkeypatch.setenv("FENIX_AMD_DEVICES", ",".join(["0"] * SHARDS))
    n = SHARDS * PER_SHARD
    x16 = np.empty((n, D), dtype=np.float16)  # generated in C block by block (12.3 GB)
    for s in range(0, n, PER_SHARD):
        x16[s : s + PER_SHARD] = O.fill_normal_c(PER_SHARD, D, 401, row_base=s)
    port = _port()
    server = fenix_amd.Server(str(tmp_path), host="127.0.0.1", port=port)
    try:
        flight = fenix_amd.Flight(host="127.0.0.1", port=port)
        flight.make_table("cfg4/source", _reader(x16))
        targets = O.fill_normal(3, D, seed=402)
        times = []
        near_ties = 0
        for i, t in enumerate(targets):
            t0 = time.perf_counter()
            r = flight.search(target=t, source="cfg4/source", column="vector",
                              metric="inner_product" if i % 2 == 0 else "dot", maxval=K)
            times.append(time.perf_counter() - t0)
            assert r.num_rows == K
            assert r.schema == pa.schema([*SCHEMA, pa.field("__DISTANCE__", pa.float16())])
            ids = r.column("id").to_numpy()
            # the query takes the column's type (index.py:101-111)
            qh = t.astype(np.float16).astype(np.float32)[None]
            od, orow = O.knn(x16, qh, "inner_product", K, threads=16)
            near_ties += _check_ids(ids, orow[0], od[0], x16, qh)
            got = r.column("__DISTANCE__").to_numpy().astype(np.float64)
            assert np.all(np.abs(got - od[0]) <= 2.0 ** -10 * np.abs(od[0]) + 2.0 ** -14)
            vec = np.stack(r.column("vector").to_numpy(zero_copy_only=False))
            np.testing.assert_array_equal(vec.view(np.uint16), x16[ids].view(np.uint16))
        # the latency a client sees: a torch-free client process, warm searches
        cmd = [sys.executable, os.path.join(ROOT, "tools", "bench_flight.py"), "--client",
               "--port", str(port), "--d", str(D), "--k", str(K), "--metric", "inner_product",
               "--dtype", "f16", "--reps", "20", "--source", "cfg4/source"]
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=ROOT)
        assert out.returncode == 0, out.stderr[-2000:]
        client = json.loads(out.stdout.strip().splitlines()[-1])
        assert client["torch_imported"] is False
        median_ms = float(np.median(client["lat_ms"]))
        # the column was staged as 8 row shards (one per listed device)
        (entry,) = [e for e in engine.CACHE._entries.values() if "cfg4" in e.key[0]]
        assert len(entry.pieces) == SHARDS
        assert [p.start for p in entry.pieces] == [g * PER_SHARD for g in range(SHARDS)]
        os.makedirs("gpurun_out", exist_ok=True)
        with open(os.path.join("gpurun_out", "cfg4_serving_test.json"), "w") as f:
            json.dump({"rows": n, "d": D, "k": K, "shards": SHARDS,
                       "client_process_lat_ms": client["lat_ms"],
                       "client_process_median_ms": median_ms,
                       "inprocess_flight_search_s": times, "near_ties": near_ties}, f)
        assert near_ties <= NEAR_TIE_CAP, near_ties
        assert median_ms <= MEDIAN_MS_BOUND, (median_ms, client["lat_ms"])
    finally:
        server.shutdown()
        engine.CACHE.clear()
