"""The result rows' vectors gathered on the device behind the scan
(engine.gather_rows / engine.search_host, used by io.index.call since
round 6) equal the stored rows, and io.index.call returns the same table
through it as through the host-side gather (io.index._gather_vectors).

The reference's take (src/fenix/io/index/index.py:166-168) returns the k
winning rows' stored embeddings; both gathers must return exactly those
bytes, for one shard, several shards on one device (row-ordered sources),
f16 columns, empty slots (n < k) and the coalesced single-query path.
"""

from __future__ import annotations

import numpy as np
import pyarrow as pa
import pytest
import torch

from fenix_amd import _lib, engine
from fenix_amd.engine import Engine, Shard
from fenix_amd.io import index, table

pytestmark = pytest.mark.gpu


def _shards(n_per, d, dtype, dev):
    eng = Engine.get(dev)
    out, base = [], 0
    for i, n in enumerate(n_per):
        x = torch.empty((n, d), dtype=dtype, device=dev)
        eng.fill(x, seed=3, row_base=base)
        out.append(Shard(x, base))
        base += n
    return out


@pytest.mark.parametrize("n_per,dtype", [([20000], torch.float32), ([7000, 5000, 9000],
                                                                     torch.float32),
                                         ([6000, 6000], torch.float16), ([30], torch.float32)])
@pytest.mark.parametrize("coalesced", [True, False])
def test_search_host_vectors_are_the_stored_rows(n_per, dtype, coalesced, monkeypatch):
    if not coalesced:
        monkeypatch.setenv("FENIX_AMD_COALESCE", "0")
    dev = torch.device("cuda", 0)
    d, k = 96, 50
    shards = _shards(n_per, d, dtype, dev)
    q = torch.from_numpy(np.random.RandomState(1).standard_normal((1, d)).astype(np.float32))
    dist, rows, vecs = engine.search_host(shards, q, _lib.METRIC_L2, k, gather=True)
    rd, rr = engine._search_all(shards, q, _lib.METRIC_L2, k)
    np.testing.assert_array_equal(rows, rr.cpu().numpy())
    np.testing.assert_array_equal(dist.view(np.uint32), rd.cpu().numpy().view(np.uint32))
    assert vecs is not None and vecs.shape == (1, k, d)
    whole = torch.cat([s.data for s in shards]).cpu().numpy()
    for j in range(k):
        r = rows[0, j]
        if r < 0:  # fewer rows than k: an empty slot, dropped by the caller
            continue
        np.testing.assert_array_equal(vecs[0, j].view(np.uint8), whole[r].view(np.uint8))
    d2, r2, v2 = engine.search_host(shards, q, _lib.METRIC_L2, k, gather=False)
    assert v2 is None
    np.testing.assert_array_equal(r2, rows)


def test_call_device_gather_equals_host_gather(tmp_path, monkeypatch):
    """io.index.call over a two-source table: the device-gathered vector
    column equals the host-side gather's, byte for byte."""
    d, n = 64, 3000
    rs = np.random.RandomState(5)
    for name, seed in (("a", 0), ("b", 1)):
        x = np.random.RandomState(seed).standard_normal((n, d)).astype(np.float32)
        arr = pa.FixedSizeListArray.from_arrays(pa.array(x.ravel()), list_size=d)
        t = pa.table({"id": pa.array(np.arange(n, dtype=np.int64)), "vector": arr})
        table.make(str(tmp_path), f"s/{name}", t.to_reader(max_chunksize=700))
    q = rs.standard_normal(d).astype(np.float32)
    got = index.call(str(tmp_path), None, ["s/a", "s/b"], "vector", q, "l2", maxval=40)

    def no_device_gather(shards, rows):
        return None

    monkeypatch.setattr(engine, "gather_rows", no_device_gather)
    ref = index.call(str(tmp_path), None, ["s/a", "s/b"], "vector", q, "l2", maxval=40)
    assert got.equals(ref)
    assert got.num_rows == 40
