"""GPU parity of the HIP kernels against the CPU oracle, through the C ABI.

Every call goes fenix_amd.engine -> ctypes -> libfenix_knn.so (gfx950);
inputs come from the portable generator (device) and are regenerated
bit-identically on the host for the oracle (oracle/knn_ref.c, float64).
"""

from __future__ import annotations

import functools
import json
import os

import numpy as np
import pytest
import torch

from fenix_amd import _lib
from fenix_amd.engine import Engine, Shard, device_mask
from oracle import oracle as O
from tests.parity import check_topk, scale_of

pytestmark = pytest.mark.gpu

METRICS = ["l2", "inner_product", "cosine"]


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return Engine.get(torch.device("cuda", 0))


def gpu_fill(eng, n, d, seed, dtype=torch.float32, row_base=0, cluster=0):
    x = torch.empty((n, d), dtype=dtype, device=eng.device)
    eng.fill(x, seed, row_base, cluster)
    return x


def gpu_search(eng, x, q, metric, k, mask=None, row_base=0):
    qt = torch.as_tensor(q, dtype=torch.float32).to(eng.device)
    m = device_mask(mask, eng.device) if mask is not None else None
    d, r = eng.search([Shard(x, row_base)], qt, _lib.METRICS[metric], k, [m])
    torch.cuda.synchronize()
    return d.cpu().numpy(), r.cpu().numpy()


# ---------------------------------------------------------------- generator


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("cluster", [0, 1000])
def test_fill_bit_exact(eng, dtype, cluster):
    n, d = 3001, 96
    x = gpu_fill(eng, n, d, seed=7, dtype=dtype, row_base=123, cluster=cluster).cpu().numpy()
    ref = O.fill_normal(n, d, 7, row_base=123, cluster=cluster,
                        dtype=np.float32 if dtype == torch.float32 else np.float16)
    assert x.tobytes() == ref.tobytes()


# ------------------------------------------------------------ golden vectors


def _golden(golden_dir, name):
    z = np.load(os.path.join(golden_dir, f"{name}.npz"))
    return z, json.loads(str(z["meta"]))


@pytest.mark.parametrize("name", ["g1_d128", "g1_d768", "g4_flight"])
def test_golden_fenix_ids_and_distances(eng, golden_dir, name):
    """GPU top-k == the reference's own io.index.call / Flight.search output."""
    z, meta = _golden(golden_dir, name)
    x = gpu_fill(eng, meta["n"], meta["d"], meta["seed"], cluster=meta["cluster"])
    q = O.fill_normal(meta["nq"], meta["d"], meta["qseed"])
    for metric in meta["metrics"]:
        for k in meta["ks"]:
            gd, gr = gpu_search(eng, x, q, metric, k)
            fid = z[f"{metric}_k{k}_ids"]
            fdist = z[f"{metric}_k{k}_dist"].astype(np.float64)
            np.testing.assert_array_equal(gr, fid, err_msg=f"{name} {metric} k={k}")
            rel = np.abs(gd - fdist) / np.abs(fdist)
            assert rel.max() <= 1e-5, f"{name} {metric} k={k}: rel {rel.max():.3e}"


def test_golden_fp16_full_table(eng, golden_dir):
    """G6 (tests/golden/g6_fp16.npz): the reference's own __DISTANCE__ column
    for a 1536-d halffloat corpus with maxval=None (index.py:150-165, ATen
    half arithmetic) against the engine's (fp16 loads, fp32 accumulation,
    rounded to halffloat) through io.index.call: within one fp16 ulp (and
    2^-14 |q||x| for inner products, tests/test_oracle_golden.fp16_tolerance),
    and within the same tolerance of the float64 oracle rounded to fp16.  The size of
    the half-accumulation difference is recorded in gpurun_out."""
    import pyarrow as pa
    from fenix_amd.io import index
    from tests.test_oracle_golden import fp16_tolerance

    z, meta = _golden(golden_dir, "g6_fp16")
    n, d = meta["n"], meta["d"]
    x = O.fill_normal(n, d, meta["seed"], dtype=np.float16)
    q = O.fill_normal(meta["nq"], d, meta["qseed"]).astype(np.float16)
    vt = pa.list_(pa.float16(), list_size=d)
    batches = [pa.record_batch([pa.array(np.arange(s, min(s + 1000, n))),
                                pa.FixedSizeListArray.from_arrays(
                                    pa.array(x[s:s + 1000].ravel()), list_size=d)],
                               names=["id", "vector"]) for s in range(0, n, 1000)]
    src = pa.Table.from_batches(batches, pa.schema({"id": pa.int64(), "vector": vt}))
    stats = {}
    for metric in meta["metrics"]:
        ref = z[f"{metric}_all_dist"]
        got = np.stack([index.call("", None, src, "vector", target=qv, metric=metric)
                        .column("__DISTANCE__").to_numpy() for qv in q])
        assert got.dtype == np.float16
        err = np.abs(got.astype(np.float64) - ref.astype(np.float64))
        tol = fp16_tolerance(ref, metric, q.astype(np.float32), x)
        assert np.all(err <= tol), (metric, float((err / tol).max()))
        o16 = O.distances(x, q.astype(np.float32), metric).astype(np.float32).astype(np.float16)
        tol64 = fp16_tolerance(o16, metric, q.astype(np.float32), x)
        assert np.all(np.abs(got.astype(np.float64) - o16.astype(np.float64)) <= tol64), metric
        stats[metric] = {"max_err_vs_reference_in_tolerance": float((err / tol).max()),
                         "frac_equal_to_reference": float((err == 0).mean()),
                         "max_abs_err_vs_reference": float(err.max())}
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "g6_fp16_stats.json"), "w") as f:
        json.dump(stats, f, indent=1)


def test_golden_ties(eng, golden_dir):
    """Duplicated rows: fenix pins the tie SET; we also pin the order (row asc)."""
    z, meta = _golden(golden_dir, "g2_ties")
    base = O.fill_normal(1024, 64, 5)
    x = torch.from_numpy(np.concatenate([base, base])).to(eng.device)
    q = O.fill_normal(meta["nq"], 64, meta["qseed"])
    for metric in meta["metrics"]:
        gd, gr = gpu_search(eng, x, q, metric, 10)
        fid = z[f"{metric}_k10_ids"]
        for i in range(len(q)):
            # same multiset of base rows (row r and r+1024 are the same vector)
            assert sorted(gr[i] % 1024) == sorted(fid[i] % 1024)
            # deterministic order: each pair appears (r, r+1024) consecutively
            for j in range(0, 10, 2):
                assert gr[i, j + 1] == gr[i, j] + 1024 and gd[i, j] == gd[i, j + 1]


def test_golden_tail_full_table(eng, golden_dir):
    """maxval >= rows: every distance in row order (index.py:165 not taken)."""
    z, meta = _golden(golden_dir, "g3_tail")
    n, d = meta["n"], meta["d"]
    x = gpu_fill(eng, n, d, meta["seed"])
    q = O.fill_normal(meta["nq"], d, meta["qseed"])
    for metric in meta["metrics"]:
        out = eng.distances(Shard(x, 0), torch.from_numpy(q), _lib.METRICS[metric])
        got = out.cpu().numpy()
        fid = z[f"{metric}_k{n}_ids"]
        fdist = z[f"{metric}_k{n}_dist"].astype(np.float64)
        np.testing.assert_array_equal(fid, np.tile(np.arange(n), (len(q), 1)))
        xh = O.fill_normal(n, d, meta["seed"])
        ref = O.distance_f64(xh, q, metric)
        sc = scale_of(xh, q, metric)[:, None]
        assert np.all(np.abs(got - ref) <= 1e-5 * np.maximum(np.abs(ref), sc))
        # and agrees with what fenix itself returned (its own f32 error included)
        assert np.all(np.abs(got - fdist) <= 1e-5 * np.maximum(np.abs(fdist), sc))


# ------------------------------------------------------- random-shape parity


CASES = [
    # n, d, k, dtype
    (1, 8, 1, torch.float32),
    (5, 3, 10, torch.float32),
    (100, 1, 7, torch.float32),
    (1000, 17, 10, torch.float32),
    (4097, 64, 100, torch.float32),
    (4097, 100, 33, torch.float32),
    (20000, 128, 10, torch.float32),
    (20000, 384, 256, torch.float32),
    (12345, 768, 100, torch.float32),
    (5000, 1000, 64, torch.float32),
    (3000, 1536, 100, torch.float32),
    (2000, 3072, 10, torch.float32),
    (20000, 768, 1000, torch.float32),
    (4097, 128, 100, torch.float16),
    (12345, 768, 100, torch.float16),
    (5000, 1536, 1000, torch.float16),
    (3001, 20, 10, torch.float16),
]


@pytest.mark.parametrize("n,d,k,dtype", CASES)
@pytest.mark.parametrize("metric", METRICS)
def test_random_parity(eng, n, d, k, dtype, metric):
    x = gpu_fill(eng, n, d, seed=n + d, dtype=dtype)
    q = O.fill_normal(3, d, seed=99)
    xh = O.fill_normal(n, d, n + d, dtype=np.float32 if dtype == torch.float32 else np.float16)
    qc = q.astype(xh.dtype).astype(np.float32)  # query cast to the column type (index.py:111)
    gd, gr = gpu_search(eng, x, qc, metric, k)
    od, orow = O.knn(xh, qc, metric, k)
    check_topk(gd, gr, od, orow, xh.astype(np.float32), qc, metric)


@pytest.mark.parametrize("metric", METRICS)
def test_mask_and_row_base(eng, metric):
    n, d, k = 30000, 256, 50
    x = gpu_fill(eng, n, d, seed=3)
    xh = O.fill_normal(n, d, 3)
    q = O.fill_normal(2, d, seed=4)
    mask = np.random.RandomState(0).rand(n) < 0.05
    gd, gr = gpu_search(eng, x, q, metric, k, mask=mask, row_base=1_000_000)
    od, orow = O.knn(xh, q, metric, k, mask=mask, row_base=1_000_000)
    check_topk(gd, gr, od, orow, xh, q, metric)
    assert mask[gr[gr >= 0] - 1_000_000].all()


def test_mask_fewer_than_k(eng):
    n, d, k = 1000, 32, 20
    x = gpu_fill(eng, n, d, seed=5)
    mask = np.zeros(n, dtype=bool)
    mask[[3, 500, 999]] = True
    gd, gr = gpu_search(eng, x, O.fill_normal(1, d, 6), "l2", k, mask=mask)
    assert sorted(gr[0, :3]) == [3, 500, 999]
    assert (gr[0, 3:] == -1).all() and np.isnan(gd[0, 3:]).all()
    gd, gr = gpu_search(eng, x, O.fill_normal(1, d, 6), "l2", k, mask=np.zeros(n, bool))
    assert (gr == -1).all()


@pytest.mark.parametrize("k", [1, 10, 100, 1000])
def test_identical_rows_select_by_row(eng, k):
    """Every distance equal: the composites differ only in their low (row)
    bytes, which drives both radix selects down to the last byte."""
    n, d = 70_000, 32
    x = torch.ones((n, d), dtype=torch.float32, device=eng.device)
    q = np.zeros((2, d), np.float32)
    for metric in METRICS:
        gd, gr = gpu_search(eng, x, q, metric, k, row_base=123)
        np.testing.assert_array_equal(gr, np.tile(np.arange(k) + 123, (2, 1)))
        assert np.all(gd == gd[0, 0])
    mask = np.zeros(n, dtype=bool)
    mask[n // 2 :] = True
    gd, gr = gpu_search(eng, x, q, "l2", k, mask=mask)
    np.testing.assert_array_equal(gr[0], np.arange(k) + n // 2)


def test_unaligned_corpus_scalar_path(eng):
    """A corpus pointer that is not 16-B aligned takes the scalar-load variant."""
    n, d, k = 5000, 64, 10
    big = gpu_fill(eng, n + 1, d, seed=8)
    flat = big.reshape(-1)[1 : 1 + n * d].view(n, d)  # 4-byte offset
    xh = O.fill_normal(n + 1, d, 8).reshape(-1)[1 : 1 + n * d].reshape(n, d)
    q = O.fill_normal(2, d, 9)
    for metric in METRICS:
        gd, gr = gpu_search(eng, flat, q, metric, k)
        od, orow = O.knn(xh, q, metric, k)
        check_topk(gd, gr, od, orow, xh, q, metric)


def test_nan_and_zero_rows(eng):
    """NaN distances order after numbers; -0/+0 tie by row; duplicates by row."""
    n, d = 300, 16
    xh = O.fill_normal(n, d, 10)
    xh[7] = np.nan
    xh[11] = np.nan
    xh[20] = 0.0
    xh[21] = -0.0
    xh[40] = xh[39]
    x = torch.from_numpy(xh).to(eng.device)
    q = O.fill_normal(1, d, 11)
    for metric in METRICS:
        gd, gr = gpu_search(eng, x, q, metric, n)
        od, orow = O.knn(xh, q, metric, n)
        check_topk(gd, gr, od, orow, np.nan_to_num(xh), q, metric)
        assert list(gr[0, -2:]) == [7, 11]
    # inner product against a zero row is -0.0 vs +0.0: must tie, broken by row
    gd, gr = gpu_search(eng, x, np.zeros((1, d), np.float32), "inner_product", n)
    zero_rows = gr[0][gd[0] == 0]
    assert list(zero_rows) == sorted(zero_rows)


def test_many_queries(eng):
    n, d, k = 20000, 128, 10
    x = gpu_fill(eng, n, d, seed=12)
    xh = O.fill_normal(n, d, 12)
    q = O.fill_normal(37, d, 13)
    for metric in METRICS:
        gd, gr = gpu_search(eng, x, q, metric, k)
        od, orow = O.knn(xh, q, metric, k)
        check_topk(gd, gr, od, orow, xh, q, metric)


@pytest.mark.parametrize("metric", METRICS)
def test_distances_kernel(eng, metric):
    n, d = 7001, 200
    x = gpu_fill(eng, n, d, seed=14)
    xh = O.fill_normal(n, d, 14)
    q = O.fill_normal(3, d, 15)
    mask = np.random.RandomState(1).rand(n) < 0.5
    got = eng.distances(Shard(x, 0), torch.from_numpy(q), _lib.METRICS[metric],
                        device_mask(mask, eng.device)).cpu().numpy()
    ref = O.distance_f64(xh, q, metric)
    sc = {"l2": 10.0, "cosine": 1.0, "inner_product": 200.0}[metric]
    ok = np.abs(got[:, mask] - ref[:, mask]) <= 1e-5 * np.maximum(np.abs(ref[:, mask]), sc)
    assert ok.all()
    assert np.isnan(got[:, ~mask]).all()


def test_topk_merge(eng):
    """fx_topk_merge == oracle top-k of the union (the multi-GPU final merge)."""
    rs = np.random.RandomState(2)
    nq, parts, kin, k = 4, 8, 50, 40
    d = rs.randn(nq, parts, kin).astype(np.float32)
    d[0, 0, :5] = d[0, 1, :5]  # cross-list exact ties -> row order
    r = np.arange(nq * parts * kin).reshape(nq, parts, kin) % 100000
    r[:, 3, 10:] = -1  # empty slots
    d[:, 3, 10:] = np.nan
    od, orow = eng.merge(torch.from_numpy(d).to(eng.device), torch.from_numpy(r).to(eng.device), k)
    od, orow = od.cpu().numpy(), orow.cpu().numpy()
    for i in range(nq):
        valid = r[i] >= 0
        dv, rv = d[i][valid], r[i][valid]
        order = np.lexsort((rv, dv))[:k]
        np.testing.assert_array_equal(orow[i], rv[order])
        np.testing.assert_array_equal(od[i], dv[order])


def test_topk_merge_non_contiguous_views(eng):
    """Engine.merge of permuted [nq, parts, k] views (the RCCL gather's
    layout, engine.DeviceComm.gather_merge): the contiguous copies must stay
    alive until the merge is queued, or the row copy can reuse the distance
    copy's block.  Repeated with fresh allocations so a reuse would show."""
    rs = np.random.RandomState(5)
    ndev, nq, k = 4, 6, 32
    for it in range(20):
        d = np.sort(rs.randn(ndev, nq, k).astype(np.float32), axis=2)
        r = (rs.permutation(ndev * nq * k).reshape(ndev, nq, k) + 7).astype(np.int64)
        td = torch.from_numpy(d).to(eng.device).permute(1, 0, 2)
        tr = torch.from_numpy(r).to(eng.device).permute(1, 0, 2)
        assert not td.is_contiguous() and not tr.is_contiguous()
        od, orow = eng.merge(td, tr, k)
        od, orow = od.cpu().numpy(), orow.cpu().numpy()
        for i in range(nq):
            dv, rv = d[:, i].ravel(), r[:, i].ravel()
            order = np.lexsort((rv, dv))[:k]
            np.testing.assert_array_equal(orow[i], rv[order])
            np.testing.assert_array_equal(od[i], dv[order])


def test_sharded_equals_whole(eng):
    """topk(all rows) == merge(topk(shard_0), topk(shard_1), ...) bit-exactly."""
    n, d, k = 60000, 768, 100
    x = gpu_fill(eng, n, d, seed=16)
    q = torch.from_numpy(O.fill_normal(2, d, 17)).to(eng.device)
    whole_d, whole_r = eng.search([Shard(x, 0)], q, 0, k)
    cuts = [0, 13331, 40000, n]
    shards = [Shard(x[a:b], a) for a, b in zip(cuts[:-1], cuts[1:])]
    sd, sr = eng.search(shards, q, 0, k)
    assert torch.equal(whole_r, sr) and torch.equal(whole_d, sd)


def test_error_paths(eng):
    x = gpu_fill(eng, 10, 8, seed=1)
    q = torch.zeros((1, 8), device=eng.device)
    with pytest.raises(NotImplementedError):
        eng.search([Shard(x, 0)], q, 0, 1 << 31)
    with pytest.raises(ValueError):
        eng.search([Shard(x, 0)], q, 7, 5)


# ------------------------------------------------------------ batched (MFMA)


@pytest.mark.parametrize("n,d,nq,k", [
    (1000, 64, 8, 10),          # n <= cap: one phase, no threshold
    (50_000, 128, 64, 10),
    (300_000, 768, 256, 100),   # three sampled phases
    (200_000, 96, 300, 1000),   # two query tiles, k = 1000
    (70_001, 36, 9, 33),        # ragged tail tile, d not a multiple of 32
])
@pytest.mark.parametrize("metric", ["l2", "inner_product", "cosine"])
def test_batched_mfma_parity(eng, n, d, nq, k, metric):
    x = gpu_fill(eng, n, d, seed=n % 97)
    xh = O.fill_normal(n, d, n % 97)
    q = O.fill_normal(nq, d, seed=5)
    gd, gr = gpu_search(eng, x, q, metric, k)
    od, orow = O.knn(xh, q, metric, k)
    check_topk(gd, gr, od, orow, xh, q, metric)


def test_batched_masked_and_clustered(eng):
    n, d, nq, k = 120_000, 256, 32, 50
    x = gpu_fill(eng, n, d, seed=3, cluster=1000)
    xh = O.fill_normal(n, d, 3, cluster=1000)
    q = O.fill_normal(nq, d, seed=4, cluster=0)
    q[:8] = xh[[5, 1500, 77_777, 119_999, 2, 3, 4, 60_000]]  # queries inside clusters
    mask = np.random.RandomState(7).rand(n) < 0.3
    for metric in ("l2", "inner_product", "cosine"):
        gd, gr = gpu_search(eng, x, q, metric, k, mask=mask, row_base=17)
        od, orow = O.knn(xh, q, metric, k, mask=mask, row_base=17)
        check_topk(gd, gr, od, orow, xh, q, metric)


def test_batched_overflow_fallback(eng):
    """Queries whose final candidates overflow are recomputed by the exact
    single-query scan (gated on the device): forced for every query, results
    must not change."""
    n, d, nq, k = 40_000, 128, 16, 20
    x = gpu_fill(eng, n, d, seed=9)
    xh = O.fill_normal(n, d, 9)
    q = O.fill_normal(nq, d, seed=10)
    ld, lr = gpu_search(eng, x, q, "l2", k)  # L2 batches: expansion filter + rescoring
    old, olr = O.knn(xh, q, "l2", k)
    check_topk(ld, lr, old, olr, xh, q, "l2")
    base_d, base_r = gpu_search(eng, x, q, "cosine", k)
    with _lib.options(force_fallback=1):
        fd, fr = gpu_search(eng, x, q, "cosine", k)
    od, orow = O.knn(xh, q, "cosine", k)
    check_topk(fd, fr, od, orow, xh, q, "cosine")
    check_topk(base_d, base_r, od, orow, xh, q, "cosine")
    np.testing.assert_array_equal(fr, base_r)
    np.testing.assert_array_equal(fd.view(np.uint32), base_d.view(np.uint32))
    with _lib.options(batch_cap=16 * k):  # tiny buffers: more phases
        sd, sr = gpu_search(eng, x, q, "cosine", k)
    check_topk(sd, sr, od, orow, xh, q, "cosine")


@pytest.mark.parametrize("k", [10, 1000])
def test_batched_overflow_fallback_rounds(eng, k):
    """The device-gated fallback runs in rounds of queries (its candidate
    lists are bounded); with every query forced through it, or only those
    whose candidates overflow a small buffer, a batch larger than a round
    equals the per-query scans bit for bit, and no call waits for the host."""
    n, d, nq = 60_000, 128, 300
    x = gpu_fill(eng, n, d, seed=13)
    q = O.fill_normal(nq, d, seed=14)
    with _lib.options(batched=0):
        sd, sr = gpu_search(eng, x, q, "l2", k)
    syncs = _lib.host_sync_count()
    for opts in ({"force_fallback": 1}, {"batch_cap": 16 * k}):
        with _lib.options(**opts):
            fd, fr = gpu_search(eng, x, q, "l2", k)
        np.testing.assert_array_equal(fr, sr)
        np.testing.assert_array_equal(fd.view(np.uint32), sd.view(np.uint32))
    assert _lib.host_sync_count() == syncs


def test_batched_equals_unbatched(eng):
    """The MFMA path and the per-query scan agree (ids; distances to f32
    rounding — and bit for bit for L2, whose candidates are rescored with the
    scan's own summation order)."""
    n, d, nq, k = 100_000, 768, 24, 100
    x = gpu_fill(eng, n, d, seed=11)
    q = O.fill_normal(nq, d, seed=12)
    xh = O.fill_normal(n, d, 11)
    for metric in ("cosine", "l2"):
        bd, br = gpu_search(eng, x, q, metric, k)
        with _lib.options(batched=0):
            sd, sr = gpu_search(eng, x, q, metric, k)
        od, orow = O.knn(xh, q, metric, k)
        check_topk(bd, br, od, orow, xh, q, metric)
        check_topk(sd, sr, od, orow, xh, q, metric)
        if metric == "l2":
            np.testing.assert_array_equal(br, sr)
            np.testing.assert_array_equal(bd, sd)
        else:
            assert np.max(np.abs(bd - sd)) <= 1e-6


@pytest.mark.parametrize("metric", METRICS)
@pytest.mark.parametrize("n,d,nq,k", [
    (100_000, 768, 40, 100),
    (30_011, 100, 300, 7),     # d not a multiple of the 32-deep K chunk
    (257, 64, 9, 300),         # n < k, a single partial tile
    (40_000, 128, 2, 50),      # the smallest batch (64-query tiles)
    (40_000, 128, 64, 50),     # the largest 64-query tile
    (40_000, 128, 65, 50),     # the smallest 128-query tile
    (40_000, 128, 128, 50),    # the largest 128-query tile
    (40_000, 128, 129, 50),    # the smallest 256-query tile
])
def test_batched_filter_bit_identical_to_scan(eng, metric, n, d, nq, k):
    """fp16-MFMA filter + exact rescoring == the single-query f32 scan, bit for
    bit (rows and distances), and both pass the oracle rule.  (The filter
    image is off here: test_filter_image_bit_identical covers it.)"""
    x = gpu_fill(eng, n, d, seed=21)
    q = O.fill_normal(nq, d, seed=22)
    with _lib.options(filter_image=0):
        fd, fr = gpu_search(eng, x, q, metric, k)
    with _lib.options(batched=0):
        sd, sr = gpu_search(eng, x, q, metric, k)
    np.testing.assert_array_equal(fr, sr)
    np.testing.assert_array_equal(fd.view(np.uint32), sd.view(np.uint32))
    xh = O.fill_normal(n, d, 21)
    od, orow = O.knn(xh, q, metric, k)
    check_topk(fd, fr, od, orow, xh, q, metric)


@pytest.mark.parametrize("dtype", ["f32", "f16"])
def test_batched_filter_sampling_plan_invariant(eng, dtype):
    """The nested sample phases only set thresholds: any candidate buffer size
    and sample ratio ("batch_cap" / "batch_sample_ratio", e.g. 2-5 phases),
    and either pass test of the sampling phases ("batch_ub_test": by upper or
    lower bound), gives the same rows and distances, bit for bit (every kept
    candidate is rescored)."""
    n, d, nq, k = 400_000, 256, 96, 50
    tdt = torch.float16 if dtype == "f16" else torch.float32
    x = gpu_fill(eng, n, d, seed=31, dtype=tdt)
    q = O.fill_normal(nq, d, seed=32)
    if dtype == "f16":
        q = q.astype(np.float16).astype(np.float32)
    for metric in METRICS:
        base_d, base_r = gpu_search(eng, x, q, metric, k)
        for cap, r, ub in ((0, 3, 1), (0, 8, 1), (32768, 0, 1), (16 * k, 2, 1), (0, 0, 0),
                           (16 * k, 2, 0), (0, 12, 0)):
            with _lib.options(batch_cap=cap, batch_sample_ratio=r, batch_ub_test=ub):
                pd, pr = gpu_search(eng, x, q, metric, k)
            np.testing.assert_array_equal(pr, base_r)
            np.testing.assert_array_equal(pd.view(np.uint32), base_d.view(np.uint32))
        with _lib.options(batched=0):
            sd, sr = gpu_search(eng, x, q, metric, k)
        np.testing.assert_array_equal(base_r, sr)
        np.testing.assert_array_equal(base_d.view(np.uint32), sd.view(np.uint32))


@pytest.mark.parametrize("metric", METRICS)
@pytest.mark.parametrize("n,d,nq,k", [(120_000, 1536, 24, 1000), (20_003, 104, 64, 10),
                                      (30_000, 200, 100, 40), (50_000, 768, 256, 100)])
def test_batched_f16_corpus_bit_identical_to_scan(eng, metric, n, d, nq, k):
    """fp16 columns (configs[4]'s dtype) in a batch: the filter reads the rows
    exactly; results equal the per-query f16 scan bit for bit."""
    x = gpu_fill(eng, n, d, seed=23, dtype=torch.float16)
    q = O.fill_normal(nq, d, seed=24).astype(np.float16).astype(np.float32)
    fd, fr = gpu_search(eng, x, q, metric, k)
    with _lib.options(batched=0):
        sd, sr = gpu_search(eng, x, q, metric, k)
    np.testing.assert_array_equal(fr, sr)
    np.testing.assert_array_equal(fd.view(np.uint32), sd.view(np.uint32))


@pytest.mark.parametrize("metric", METRICS)
def test_batched_filter_extreme_rows_and_queries(eng, metric):
    """Rows the fp16 filter cannot bound (|x| >= 65504, inf, NaN) are forced
    through; tiny-magnitude rows and queries scaled by 2^+-60 still bound
    correctly: results equal the scan's bit for bit."""
    n, d, k = 20_000, 64, 25
    xh = O.fill_normal(n, d, 31)
    rs = np.random.RandomState(5)
    big = rs.choice(n, 40, replace=False)
    xh[big[:10]] *= 1e5                    # beyond fp16 range
    xh[big[10:20]] *= 1e-7                 # fp16 subnormal / flushed range
    xh[big[20:25], 3] = np.inf
    xh[big[25:30], 7] = np.nan
    xh[big[30:35]] = 0.0
    xh[big[35:40]] *= 3e4                  # just below fp16 max
    x = torch.from_numpy(xh).to(eng.device)
    q = O.fill_normal(16, d, seed=32)
    q[0] *= 2.0 ** 60
    q[1] *= 2.0 ** -60
    q[2] = xh[big[0]]                      # a query out of fp16 range
    q[3] = xh[big[12]]                     # a tiny query
    q[4] = 0.0
    for image in (8, 16, 0):
        with _lib.options(filter_image=image):
            fd, fr = gpu_search(eng, x, q, metric, k)
        with _lib.options(batched=0):
            sd, sr = gpu_search(eng, x, q, metric, k)
        bad = np.nonzero((fr != sr).any(axis=1))[0]
        np.testing.assert_array_equal(fr, sr, err_msg=f"image {image}: queries {bad}")
        np.testing.assert_array_equal(fd.view(np.uint32), sd.view(np.uint32))


@pytest.mark.parametrize("metric", METRICS)
def test_batched_f16_extreme_rows_and_queries(eng, metric):
    """fp16 columns with +-inf, NaN, zero, subnormal and near-max rows, and
    queries scaled by 2^+-40: the batched path equals the scan."""
    n, d, k = 20_000, 64, 25
    xh = O.fill_normal(n, d, 33).astype(np.float16)
    rs = np.random.RandomState(6)
    sel = rs.choice(n, 40, replace=False)
    xh[sel[:10]] = (xh[sel[:10]].astype(np.float32) * 1e-6).astype(np.float16)  # subnormal
    xh[sel[10:15], 3] = np.inf
    xh[sel[15:20], 5] = -np.inf
    xh[sel[20:25], 7] = np.nan
    xh[sel[25:30]] = 0.0
    xh[sel[30:40]] = (np.sign(xh[sel[30:40]].astype(np.float32)) * 60000.0).astype(np.float16)
    x = torch.from_numpy(xh).to(eng.device)
    q = O.fill_normal(16, d, seed=34).astype(np.float16).astype(np.float32)
    q[0] *= 2.0 ** 40
    q[1] *= 2.0 ** -40
    q[2] = xh[sel[35]].astype(np.float32)  # a near-max query
    q[3] = xh[sel[2]].astype(np.float32)   # a subnormal query
    q[4] = 0.0
    fd, fr = gpu_search(eng, x, q, metric, k)
    with _lib.options(batched=0):
        sd, sr = gpu_search(eng, x, q, metric, k)
    np.testing.assert_array_equal(fr, sr)
    np.testing.assert_array_equal(fd.view(np.uint32), sd.view(np.uint32))


# ------------------------------------------------------- fp16 filter image


def _extreme_rows(n, d, seed):
    xh = O.fill_normal(n, d, seed)
    rs = np.random.RandomState(seed)
    sel = rs.choice(n, 48, replace=False)
    xh[sel[:8]] *= 1e5                      # beyond fp16 range: forced through
    xh[sel[8:16]] *= 1e-7                   # fp16 subnormal range
    xh[sel[16:20], 3] = np.inf
    xh[sel[20:24], 7] = np.nan
    xh[sel[24:28]] = 0.0
    xh[sel[28:36]] *= 3e4                   # just below fp16 max
    xh[sel[36:40], 5] = 65519.0             # rounds to 65504: finite
    xh[sel[40:44], 5] = 65520.0             # rounds to infinity: forced
    xh[sel[44:48], 1] = -np.inf
    return xh


@functools.lru_cache(maxsize=4)
def _extreme_rows_cached(n, d, seed):
    """(one generation per shape across the metric parametrisations)"""
    return _extreme_rows(n, d, seed)


def _build_image(x, n, d):
    """fx_filter_image into buffers of fx_filter_image_bytes."""
    import ctypes
    ib, rb = ctypes.c_size_t(0), ctypes.c_size_t(0)
    _lib.check(_lib.load().fx_filter_image_bytes(n, d, ctypes.byref(ib), ctypes.byref(rb)))
    img = torch.empty((ib.value // 2,), dtype=torch.float16, device=x.device)
    info = torch.empty((n,), dtype=torch.float32, device=x.device)
    _lib.check(_lib.load().fx_filter_image(x.data_ptr(), n, d, img.data_ptr(), info.data_ptr(),
                                           torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    return img, info


def _image_rows(img, n, d):
    """[n, d] fp16 rows of a filter image in the MFMA-fragment layout
    [tile][k-step][lane half][row in tile][8] (padding zero)."""
    h = img.cpu().numpy()
    t, ks = (n + 31) // 32, (d + 15) // 16
    full = h.reshape(t, ks, 2, 32, 8).transpose(0, 3, 1, 2, 4).reshape(t * 32, ks * 16)
    assert not full[n:].any() and not full[:, d:].any(), "image padding is not zero"
    return full[:n, :d]


def test_filter_image_contents(eng):
    """fx_filter_image: each component rounded to nearest-even fp16 (torch's
    own conversion, bit for bit, infinities included), rowinfo = the row's sum
    of squares (float64 reference, 1e-5), NaN exactly for the rows the filter
    must force through (non-finite, or a component >= 65520)."""
    n, d = 5_003, 136
    xh = _extreme_rows(n, d, 41)
    x = torch.from_numpy(xh).to(eng.device)
    img, info = _build_image(x, n, d)
    want = x.half().cpu().numpy().view(np.uint16)
    np.testing.assert_array_equal(_image_rows(img, n, d).view(np.uint16), want)
    got = info.cpu().numpy()
    with np.errstate(over="ignore", invalid="ignore"):
        ss = np.sum(xh.astype(np.float64) ** 2, axis=1)
        forced = ~np.isfinite(ss) | (ss > 3.4e38) | (np.nanmax(np.abs(xh), axis=1) >= 65520.0)
    forced |= np.isnan(xh).any(axis=1)
    np.testing.assert_array_equal(np.isnan(got), forced)
    np.testing.assert_allclose(got[~forced], ss[~forced], rtol=1e-5, atol=1e-30)
    # argument checks: d not a multiple of 8, misaligned image
    rc = _lib.load().fx_filter_image(x.data_ptr(), n, 100, img.data_ptr(), info.data_ptr(), None)
    assert rc != 0
    rc = _lib.load().fx_filter_image(x.data_ptr(), n, d, img.data_ptr() + 2, info.data_ptr(), None)
    assert rc != 0


def _build_image8(x, n, d):
    """fx_filter_image8 into buffers of fx_filter_image8_bytes."""
    import ctypes
    ib, rb = ctypes.c_size_t(0), ctypes.c_size_t(0)
    _lib.check(_lib.load().fx_filter_image8_bytes(n, d, ctypes.byref(ib), ctypes.byref(rb)))
    assert ib.value == (n + 31) // 32 * ((d + 31) // 32) * 1024 and rb.value == n * 16
    img = torch.empty((ib.value,), dtype=torch.uint8, device=x.device)
    info = torch.empty((n, 4), dtype=torch.float32, device=x.device)
    _lib.check(_lib.load().fx_filter_image8(x.data_ptr(), n, d, img.data_ptr(), info.data_ptr(),
                                            torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    return img, info


def test_filter_image8_contents(eng):
    """fx_filter_image8: rows in the int8 MFMA-fragment layout [tile][k-step]
    [lane half][row in tile][16], in the permuted row order
    (fx_filter_image8_perm); per row x~ = rint(x / s) with |x~| <= 127,
    |x~| <= 2048, every component within s/2 of x / s, and the bound terms
    {omega, 1/s, N/s, n^2/s}: omega >= |x~| + kappa |x - s x~| / s (float64
    reference), NaN exactly for non-finite rows, 0 for zero rows."""
    n, d = 5_003, 136
    xh = _extreme_rows(n, d, 41)
    x = torch.from_numpy(xh).to(eng.device)
    img, info = _build_image8(x, n, d)
    h = img.cpu().numpy().view(np.int8)
    t, ks = (n + 31) // 32, (d + 31) // 32
    full = h.reshape(t, ks, 2, 32, 16).transpose(0, 3, 1, 2, 4).reshape(t * 32, ks * 32)
    assert not full[n:].any() and not full[:, d:].any(), "image padding is not zero"
    # image row i holds corpus row (mult * i) % n (fx_filter_image8_perm):
    # back to corpus order
    perm = (_lib.image8_perm(n) * np.arange(n, dtype=np.int64)) % n
    xq = np.empty((n, d))
    xq[perm] = full[:n, :d].astype(np.float64)
    inf = np.empty((n, 4))
    inf[perm] = info.cpu().numpy().astype(np.float64)
    om, is_, nos, n2s = inf.T
    with np.errstate(over="ignore", invalid="ignore"):
        forced = ~np.isfinite(xh).all(axis=1)
    np.testing.assert_array_equal(np.isnan(om), forced)
    ok = ~forced
    zero = ok & ~xh.any(axis=1)
    assert (om[zero] == 0).all() and not xq[zero].any()
    live = ok & ~zero
    s = 1.0 / is_[live]
    x64 = xh[live].astype(np.float64)
    res = x64 - s[:, None] * xq[live]
    assert (np.abs(xq) <= 127).all()
    w = np.sqrt((xq[live] ** 2).sum(axis=1))
    assert (w <= 2048).all()
    assert (np.abs(res) <= 0.5 * s[:, None] * (1 + 1e-5)).all()
    e = np.sqrt((res ** 2).sum(axis=1))
    assert (om[live] >= w + 128.0 * e / s).all()
    assert (om[live] <= (w + 128.0 * e / s) * (1 + 1e-4) + 1e-3).all()
    nrm = np.sqrt((x64 ** 2).sum(axis=1))
    np.testing.assert_allclose(nos[live], np.maximum(nrm, 1e-12) / s, rtol=1e-5)
    np.testing.assert_allclose(n2s[live], nrm ** 2 / s, rtol=1e-5)
    # argument checks: d not a multiple of 8, misaligned image
    rc = _lib.load().fx_filter_image8(x.data_ptr(), n, 100, img.data_ptr(), info.data_ptr(), None)
    assert rc != 0
    rc = _lib.load().fx_filter_image8(x.data_ptr(), n, d, img.data_ptr() + 2, info.data_ptr(),
                                      None)
    assert rc != 0


@pytest.mark.parametrize("bits", [8, 16])
@pytest.mark.parametrize("metric", METRICS)
@pytest.mark.parametrize("n,d,nq,k", [(100_000, 768, 40, 100), (60_000, 256, 256, 64),
                                      (30_000, 64, 2, 300), (20_000, 136, 70, 25)])
def test_filter_image_bit_identical(eng, metric, n, d, nq, k, bits):
    """Batched f32 searches through the int8 (the default) and the fp16
    filter images equal the same searches without one
    (option filter_image=0) and the single-query scan, bit for bit, over
    rows the images cannot represent (beyond fp16 range, infinities, NaN,
    subnormal, zero)."""
    xh = _extreme_rows(n, d, 43)
    x = torch.from_numpy(xh).to(eng.device)
    q = O.fill_normal(nq, d, seed=44)
    q[0] *= 2.0 ** 50
    q[min(1, nq - 1)] = xh[7] if nq > 1 else q[0]
    eng.clear_images()
    with _lib.options(filter_image=bits):
        # (int8 images serve k <= option i8_max_k, 1 024 by default)
        used = _lib.filter_image_used(n, d, _lib.DTYPE_F32, nq, k, _lib.METRICS[metric])
        assert used == (bits == 16 or k <= _lib.get_option("i8_max_k"))
        id_, ir = gpu_search(eng, x, q, metric, k)  # MFMA-fragment-order image
    if used:
        assert eng._images[id(x)][0][3] == bits  # the image path ran
    else:
        assert id(x) not in eng._images
    eng.clear_images()
    with _lib.options(filter_image=0):
        nd, nr = gpu_search(eng, x, q, metric, k)
    with _lib.options(batched=0):
        sd, sr = gpu_search(eng, x, q, metric, k)
    for dd, rr in ((id_, ir), (nd, nr)):
        np.testing.assert_array_equal(rr, sr)
        np.testing.assert_array_equal(dd.view(np.uint32), sd.view(np.uint32))


@pytest.mark.parametrize("bits", [8, 16])
@pytest.mark.parametrize("metric", METRICS)
def test_single_query_through_filter_image(eng, metric, bits):
    """"batch_min_queries" = 1: single queries take the batched filter over
    the image (64-query tiles, one live query) and still equal the scan bit
    for bit, also through the overflow fallback ("force_fallback": the
    single query rescanned at the full scan's width).  By default a single
    query takes the int8 image only over a >= 4 GiB f32 or f16 corpus
    ("single_query_image")."""
    n, d, k = 80_000, 256, 100
    xh = _extreme_rows(n, d, 45)
    x = torch.from_numpy(xh).to(eng.device)
    eng.clear_images()
    with _lib.options(batch_min_queries=1, filter_image=bits):
        assert _lib.filter_image_used(n, d, _lib.DTYPE_F32, 1, k, _lib.METRICS[metric])
        for seed in (46, 47):
            q = O.fill_normal(1, d, seed=seed)
            fd, fr = gpu_search(eng, x, q, metric, k)
            with _lib.options(batched=0):
                sd, sr = gpu_search(eng, x, q, metric, k)
            np.testing.assert_array_equal(fr, sr)
            np.testing.assert_array_equal(fd.view(np.uint32), sd.view(np.uint32))
            with _lib.options(force_fallback=1):
                gd, gr = gpu_search(eng, x, q, metric, k)
            np.testing.assert_array_equal(gr, sr)
            np.testing.assert_array_equal(gd.view(np.uint32), sd.view(np.uint32))
    assert not _lib.filter_image_used(n, d, _lib.DTYPE_F32, 1, k, _lib.METRICS[metric])
    m = _lib.METRICS[metric]
    big = (10_000_000, 768)  # 30.7 GB: >= 4 GiB
    assert _lib.filter_image_used(*big, _lib.DTYPE_F32, 1, k, m)  # (defaults: int8 image)
    with _lib.options(filter_image=16):
        assert not _lib.filter_image_used(*big, _lib.DTYPE_F32, 1, k, m)
    with _lib.options(single_query_image=0):
        assert not _lib.filter_image_used(*big, _lib.DTYPE_F32, 1, k, m)
    # an fp16 column takes the int8 image too (>= 4 GiB of fp16 rows), never an fp16 image
    assert _lib.filter_image_used(*big, _lib.DTYPE_F16, 1, k, m)
    # k = 1 000 (configs[4]) takes the int8 image too (i8_max_k 1 024,
    # profiles/r06_k1000_sweep.json); k above i8_max_k does not
    assert _lib.get_option("i8_max_k") == 1024
    assert _lib.filter_image_used(*big, _lib.DTYPE_F16, 1, 1000, m)
    assert _lib.filter_image_used(*big, _lib.DTYPE_F32, 1, 1000, m)
    with _lib.options(i8_max_k=256):
        assert not _lib.filter_image_used(*big, _lib.DTYPE_F16, 1, 1000, m)
        assert not _lib.filter_image_used(*big, _lib.DTYPE_F32, 1, 1000, m)
    with _lib.options(filter_image=16):
        assert not _lib.filter_image_used(*big, _lib.DTYPE_F16, 1, k, m)


@pytest.mark.parametrize("metric", METRICS)
def test_img6_resident_slices_equal_streamed_tile(eng, metric):
    """Int8-image batches of up to 128 queries (single queries included) run
    the resident-query-slice kernel (option "img6": 64- or 128-query slices
    in LDS; with img6 = 2 larger batches too, their slices on CUs sharing the
    tiles); the same products, pass test and bounds as the streamed-tile
    kernel, so the same candidate counts and results bit for bit, equal to
    the exact scan -- across the 64 / 128 / 256 slice edges, with rows the
    image cannot represent and with a mask."""
    n, d, k = 70_000, 136, 30
    xh = _extreme_rows(n, d, 49)
    x = torch.from_numpy(xh).to(eng.device)
    eng.clear_images()
    mask = np.random.RandomState(4).rand(n) < 0.8
    m = _lib.METRICS[metric]
    for nq in (1, 2, 3, 7, 64, 65, 128, 129, 256, 300):
        qh = O.fill_normal(nq, d, seed=60 + nq)
        qh[min(3, nq - 1)] = xh[17] * 2.0
        q = torch.from_numpy(qh).to(eng.device)
        for msk in (None, mask):
            dm = device_mask(msk, eng.device) if msk is not None else None
            got = {}
            for img6 in (2, 0):
                with _lib.options(img6=img6, filter_image=8, batch_min_queries=1):
                    st = eng.scan(Shard(x, 0), q, m, k, dm)
                    counts, cap = eng.filter_counts(Shard(x, 0), nq, m, k, st)
                    od = torch.empty((nq, k), dtype=torch.float32, device=eng.device)
                    orow = torch.empty((nq, k), dtype=torch.int64, device=eng.device)
                    eng.reduce(Shard(x, 0), q, m, k, st, od, orow, dm)
                    got[img6] = (counts, od.cpu().numpy(), orow.cpu().numpy())
            assert got[2][0] is not None
            np.testing.assert_array_equal(got[2][0], got[0][0], err_msg=f"nq {nq} mask {msk is not None}")
            np.testing.assert_array_equal(got[2][2], got[0][2])
            np.testing.assert_array_equal(got[2][1].view(np.uint32), got[0][1].view(np.uint32))
            with _lib.options(batched=0):
                sd, sr = gpu_search(eng, x, qh, metric, k, mask=msk)
            np.testing.assert_array_equal(got[2][2], sr)
            np.testing.assert_array_equal(got[2][1].view(np.uint32), sd.view(np.uint32))
    eng.clear_images()


@pytest.mark.parametrize("metric", METRICS)
@pytest.mark.parametrize("d", [40, 136, 300, 768])
def test_img8_queries_in_registers_equal_streamed_tile(eng, metric, d):
    """Int8-image batches of more than 128 queries with d <= 768 run
    filter_img8_kernel (option "img8": the queries as MFMA A operands in
    registers, the image through an LDS-DMA ring, 8-byte append entries
    bounded at the flush) for every phase but the all-pass first sample; the
    same integer products, the same f32 pass test per (row, query) pair and
    the same bounds as filter_img3_kernel, so the same candidate counts and
    results bit for bit, equal to the exact scan -- over partial query tiles
    (129, 300), ring chunks per tile odd (d 40: 1, d 300: 3; one barrier per
    chunk) and even (136: 2 with a partial last chunk, 768: 6; one per
    pair), rows the image cannot represent and a mask.  600 000 rows make a
    three-phase plan (19, 293, 2 344 tiles): the all-pass first sample, F1
    and F2 all run the kernel (a one- or two-phase plan's all-pass F1 keeps
    both bounds and stays with the appending kernels)."""
    n, k = 600_000, 30
    xh = _extreme_rows_cached(n, d, 81)
    x = torch.from_numpy(xh).to(eng.device)
    eng.clear_images()
    mask = np.random.RandomState(82).rand(n) < 0.8
    m = _lib.METRICS[metric]
    for nq in (129, 256, 300):
        qh = O.fill_normal(nq, d, seed=83 + nq)
        qh[3] = xh[17] * 2.0
        q = torch.from_numpy(qh).to(eng.device)
        for msk in (None, mask):
            dm = device_mask(msk, eng.device) if msk is not None else None
            got = {}
            for img8 in (1, 0):
                with _lib.options(img8=img8, filter_image=8):
                    st = eng.scan(Shard(x, 0), q, m, k, dm)
                    counts, cap = eng.filter_counts(Shard(x, 0), nq, m, k, st)
                    od = torch.empty((nq, k), dtype=torch.float32, device=eng.device)
                    orow = torch.empty((nq, k), dtype=torch.int64, device=eng.device)
                    eng.reduce(Shard(x, 0), q, m, k, st, od, orow, dm)
                    got[img8] = (counts, od.cpu().numpy(), orow.cpu().numpy())
            assert got[1][0] is not None
            np.testing.assert_array_equal(got[1][0], got[0][0], err_msg=f"nq {nq} mask {msk is not None}")
            np.testing.assert_array_equal(got[1][2], got[0][2])
            np.testing.assert_array_equal(got[1][1].view(np.uint32), got[0][1].view(np.uint32))
            with _lib.options(batched=0):
                sd, sr = gpu_search(eng, x, qh, metric, k, mask=msk)
            np.testing.assert_array_equal(got[1][2], sr)
            np.testing.assert_array_equal(got[1][1].view(np.uint32), sd.view(np.uint32))
    eng.clear_images()


@pytest.mark.parametrize("metric", METRICS)
def test_small_batches_rescore_all_and_fallback_lists(eng, metric):
    """One or two queries through the int8 image skip the final exact
    threshold and rescore every candidate under F1's (rescore_dense_kernel);
    an overflowing query's exact-scan lists feed the final select directly
    (no merge levels).  With a mask, forced through the fallback or not, the
    results equal the exact scan bit for bit, at 1, 2 and 3 queries (either
    side of both switches)."""
    n, d, k = 90_000, 192, 50
    xh = _extreme_rows(n, d, 71)
    x = torch.from_numpy(xh).to(eng.device)
    eng.clear_images()
    mask = np.random.RandomState(72).rand(n) < 0.7
    for nq in (1, 2, 3):
        qh = O.fill_normal(nq, d, seed=73 + nq)
        for msk in (None, mask):
            with _lib.options(batched=0):
                sd, sr = gpu_search(eng, x, qh, metric, k, mask=msk)
            with _lib.options(batch_min_queries=1, filter_image=8):
                assert _lib.filter_image_used(n, d, _lib.DTYPE_F32, nq, k, _lib.METRICS[metric])
                fd, fr = gpu_search(eng, x, qh, metric, k, mask=msk)
                with _lib.options(force_fallback=1):
                    gd, gr = gpu_search(eng, x, qh, metric, k, mask=msk)
            for dd, rr in ((fd, fr), (gd, gr)):
                np.testing.assert_array_equal(rr, sr)
                np.testing.assert_array_equal(dd.view(np.uint32), sd.view(np.uint32))
    eng.clear_images()


@pytest.mark.parametrize("img6", [0, 1, 2])
def test_filter_candidate_counts_repeat_exactly(eng, img6):
    """The same int8-image search repeated appends exactly the same
    candidates: a kernel that reads a product, a query chunk or a row term
    before it has landed shows up as counts moving between identical runs
    long before it moves a result (tools/race_check.py; the resident-slice
    kernel without its pre-epilogue barrier moved in 201 of 232 repetitions,
    DESIGN.md 3.6d item 7).  nq 1-64 run the q64i build (img6 1 and 2: its
    resident-slice kernel, configs[1]'s product default for a single query),
    65 the q128 build, 256 and 300 the queries-in-registers kernel
    (filter_img8_kernel) or two slices;
    batch_min_queries=1 sends the single query through the filter."""
    n, d, k = 70_000, 768, 30
    x = torch.from_numpy(_extreme_rows(n, d, 49)).to(eng.device)
    eng.clear_images()
    for nq in (1, 2, 16, 64, 65, 256, 300):
        q = torch.from_numpy(O.fill_normal(nq, d, seed=60 + nq)).to(eng.device)
        with _lib.options(img6=img6, filter_image=8, batch_min_queries=1):
            ref = None
            for _ in range(8):
                st = eng.scan(Shard(x, 0), q, _lib.METRICS["l2"], k)
                c, _cap = eng.filter_counts(Shard(x, 0), nq, _lib.METRICS["l2"], k, st)
                assert c is not None
                if ref is None:
                    ref = c
                np.testing.assert_array_equal(c, ref, err_msg=f"nq {nq}: counts moved")
    eng.clear_images()


def test_filter_image_follows_corpus_changes(eng):
    """The cached image is keyed on the corpus tensor's version: an in-place
    torch update and a rewrite through Engine.fill both rebuild it, so the
    batched results keep equalling the scan's."""
    n, d, nq, k = 50_000, 128, 32, 20
    x = gpu_fill(eng, n, d, seed=51)
    q = O.fill_normal(nq, d, seed=52)
    gpu_search(eng, x, q, "l2", k)
    first = eng._images[id(x)][1]
    for change in (lambda: x.mul_(-0.5), lambda: eng.fill(x, 53)):
        change()
        bd, br = gpu_search(eng, x, q, "l2", k)
        assert eng._images[id(x)][1] is not first
        first = eng._images[id(x)][1]
        with _lib.options(batched=0):
            sd, sr = gpu_search(eng, x, q, "l2", k)
        np.testing.assert_array_equal(br, sr)
        np.testing.assert_array_equal(bd.view(np.uint32), sd.view(np.uint32))
    key = id(x)
    del x
    import gc
    gc.collect()
    assert key not in eng._images


# ---------------------------------------------------------------- row lists


@pytest.mark.parametrize("n,frac", [(1, 1.0), (1000, 0.3), (100_003, 0.01), (300_000, 0.45)])
def test_mask_compact_is_ordered_nonzero(eng, n, frac):
    rs = np.random.RandomState(n)
    keep = rs.rand(n) < frac
    m = device_mask(keep, eng.device)
    with eng.lock:
        rows, cnt = eng.compact(m, n)
    torch.cuda.synchronize()
    c = int(cnt.item())
    assert c == int(keep.sum())
    np.testing.assert_array_equal(rows.cpu().numpy()[:c], np.nonzero(keep)[0])


@pytest.mark.parametrize("metric", METRICS)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_row_list_search_equals_masked_search(eng, metric, dtype):
    """fx_knn_search_rows over the compacted rows == the masked full scan,
    bit for bit, and == the oracle over the kept rows."""
    n, d, k = 200_000, 96, 50
    x = gpu_fill(eng, n, d, seed=61, dtype=dtype, row_base=0, cluster=1000)
    q = O.fill_normal(2, d, seed=62)
    keep = np.random.RandomState(5).rand(n) < 0.05
    qt = torch.from_numpy(q).to(eng.device)
    m = device_mask(keep, eng.device)
    mid = _lib.METRICS[metric]
    d_mask, r_mask = eng.search([Shard(x, 1000)], qt, mid, k, [m])
    d_rows, r_rows = eng.search([Shard(x, 1000)], qt, mid, k, [m], [int(keep.sum())])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(r_rows.cpu().numpy(), r_mask.cpu().numpy())
    np.testing.assert_array_equal(d_rows.cpu().numpy(), d_mask.cpu().numpy())
    xh = O.fill_normal(n, d, 61, cluster=1000,
                       dtype=np.float32 if dtype == torch.float32 else np.float16)
    od, orow = O.knn(xh.astype(np.float32), q, metric, k, mask=keep)
    check_topk(d_rows.cpu().numpy(), r_rows.cpu().numpy() - 1000, od, orow, xh.astype(np.float32),
               q, metric)


def test_row_list_search_empty_and_all(eng):
    n, d, k = 5000, 32, 10
    x = gpu_fill(eng, n, d, seed=63)
    qt = torch.from_numpy(O.fill_normal(1, d, seed=64)).to(eng.device)
    none = device_mask(np.zeros(n, bool), eng.device)
    dd, rr = eng.search([Shard(x, 0)], qt, _lib.METRIC_L2, k, [none], [0])
    torch.cuda.synchronize()
    assert np.all(rr.cpu().numpy() == -1) and np.all(np.isnan(dd.cpu().numpy()))
    one = np.zeros(n, bool)
    one[1234] = True
    dd, rr = eng.search([Shard(x, 0)], qt, _lib.METRIC_L2, k,
                        [device_mask(one, eng.device)], [1])
    torch.cuda.synchronize()
    assert rr.cpu().numpy()[0, 0] == 1234 and np.all(rr.cpu().numpy()[0, 1:] == -1)


# ---------------------------------------------------------------- RCCL exchange


def test_rccl_allgather_single_device(eng):
    """fx_comm_init_all / fx_allgather_topk with one rank (the box has one GPU;
    the N-rank layout is [ndev][nq][k]) and the merge that follows."""
    from fenix_amd.engine import DeviceComm

    comm = DeviceComm([eng.device])
    try:
        d = torch.from_numpy(np.sort(np.random.RandomState(0).rand(3, 7).astype(np.float32), 1))
        r = torch.arange(21, dtype=torch.int64).reshape(3, 7)
        d, r = d.to(eng.device), r.to(eng.device)
        (ad, ar), = comm.allgather([(d, r)])
        torch.cuda.synchronize()
        assert ad.shape == (1, 3, 7)
        np.testing.assert_array_equal(ad[0].cpu().numpy(), d.cpu().numpy())
        np.testing.assert_array_equal(ar[0].cpu().numpy(), r.cpu().numpy())
        md, mr = comm.gather_merge([(d, r)], 5)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mr.cpu().numpy(), r.cpu().numpy()[:, :5])
    finally:
        comm.close()


# ---------------------------------------------------------------- k > 1024


@pytest.mark.parametrize("metric", METRICS)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_large_k_sorted_path(eng, metric, dtype):
    """k above the fused path's 1024 (the reference's maxval is unbounded):
    distance-mode scan + radix sort, same results as the oracle."""
    n, d, k = 20_000, 64, 3000
    x = gpu_fill(eng, n, d, seed=81, dtype=dtype)
    q = O.fill_normal(3, d, seed=82)
    xh = O.fill_normal(n, d, 81, dtype=np.float32 if dtype == torch.float32 else np.float16)
    xh = xh.astype(np.float32)
    gd, gr = gpu_search(eng, x, q, metric, k, row_base=0)
    od, orow = O.knn(xh, q, metric, k)
    check_topk(gd, gr, od, orow, xh, q, metric)
    keep = np.random.RandomState(2).rand(n) < 0.3  # masked; < 50 %: row-list path
    gd, gr = gpu_search(eng, x, q, metric, 2500, mask=keep)
    od, orow = O.knn(xh, q, metric, 2500, mask=keep)
    check_topk(gd, gr, od, orow, xh, q, metric)
    m = device_mask(keep, eng.device)
    d2, r2 = eng.search([Shard(x, 0)], torch.from_numpy(q).to(eng.device), _lib.METRICS[metric],
                        2500, [m], [int(keep.sum())])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(r2.cpu().numpy(), gr)


def test_large_k_exceeding_rows_and_multi_shard_merge(eng):
    n, d = 1500, 32
    x = gpu_fill(eng, n, d, seed=83)
    q = O.fill_normal(1, d, seed=84)
    gd, gr = gpu_search(eng, x, q, "l2", 2000)
    assert np.all(gr[0, n:] == -1) and np.all(np.isnan(gd[0, n:]))
    np.testing.assert_array_equal(np.sort(gr[0, :n]), np.arange(n))
    # three shards, k = 2500 > each shard: merged by the sort-based fx_topk_merge
    big = gpu_fill(eng, 9000, d, seed=85)
    shards = [Shard(big[0:3000], 0), Shard(big[3000:6000], 3000), Shard(big[6000:], 6000)]
    qt = torch.from_numpy(q).to(eng.device)
    dd, rr = eng.search(shards, qt, _lib.METRIC_IP, 2500)
    torch.cuda.synchronize()
    od, orow = O.knn(O.fill_normal(9000, d, 85), q, "inner_product", 2500)
    check_topk(dd.cpu().numpy(), rr.cpu().numpy(), od, orow, O.fill_normal(9000, d, 85), q,
               "inner_product")


# ------------------------------------------------- scan partitions (round 2)


@pytest.mark.parametrize("n,d,dtype", [(37, 768, torch.float32), (50_000, 768, torch.float32),
                                       (200_003, 1536, torch.float16), (80_001, 256, torch.float32),
                                       (70_000, 1000, torch.float32)])
@pytest.mark.parametrize("metric", METRICS)
def test_interleaved_scan_equals_contiguous(eng, n, d, dtype, metric):
    """Block steps dealt round-robin over the grid ("scan_interleave" 1, the
    default for rows of >= 1 KB) and one contiguous range per block give the
    same top-k bit for bit: unmasked, masked, row-list scans, several single
    queries per launch ("batched" 0), and distance mode."""
    x = gpu_fill(eng, n, d, seed=71, dtype=dtype, cluster=500)
    q = torch.from_numpy(O.fill_normal(3, d, seed=72)).to(eng.device)
    keep = np.random.RandomState(7).rand(n) < 0.3
    m = device_mask(keep, eng.device)
    mid = _lib.METRICS[metric]
    k = min(64, n)
    out = {}
    for il in (0, 1):
        with _lib.options(batched=0, scan_interleave=il):
            res = [eng.search([Shard(x, 11)], q, mid, k),
                   eng.search([Shard(x, 11)], q, mid, k, [m]),
                   eng.search([Shard(x, 11)], q, mid, k, [m], [int(keep.sum())]),
                   (eng.distances(Shard(x, 11), q, mid),)]
            torch.cuda.synchronize()
        out[il] = [tuple(t.cpu().numpy() for t in r) for r in res]
    ref = out[0]
    for key, got in out.items():
        for a, b in zip(ref, got):
            for ta, tb in zip(a, b):
                np.testing.assert_array_equal(ta.view(np.uint8), tb.view(np.uint8), err_msg=str(key))
    # and the unmasked result is the oracle's
    xh = O.fill_normal(n, d, 71, cluster=500,
                       dtype=np.float32 if dtype == torch.float32 else np.float16).astype(np.float32)
    od, orow = O.knn(xh, q.cpu().numpy(), metric, k)
    check_topk(ref[0][0], ref[0][1] - 11, od, orow, xh, q.cpu().numpy(), metric)


# ---------------------------------------- several shards on one device, one merge


@pytest.mark.parametrize("metric", METRICS)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.uint8])
def test_search_shards_one_merge_equals_per_shard(eng, metric, dtype):
    """fx_knn_search_shards (every shard's scan into one list buffer, ONE
    merge tree) returns the per-shard form's bits (a merge per shard, then
    fx_topk_merge over the shards), and the oracle's rows: shards of uneven
    sizes, one smaller than k, one 4 bytes off 16-byte alignment (the
    scalar-load scan), row bases with gaps (global rows of the sources as
    numbered by table.py:19-21), k from 10 to the fused scan's 1 024.
    uint8: quint8 code shards (FX_DTYPE_QU8), each with its own
    scale and zero point, all 16-B aligned; the oracle scans the dequantised
    values (quint8.py:53-54)."""
    d = 136
    sizes = [50_000, 777, 20_000, 3_001]
    xs, shards, base = [], [], 0
    if dtype == torch.uint8:
        for i, n in enumerate(sizes):
            codes = np.random.RandomState(80 + i).randint(0, 128, size=(n, d)).astype(np.uint8)
            scale, zp = float(np.float32(0.03 + 0.01 * i)), 60 + i
            xs.append(O.dequantize(codes, scale, zp).astype(np.float32))
            shards.append(Shard(torch.from_numpy(codes).to(eng.device), base, scale, zp))
            base += n + 1000 * (i + 1)
    for i, n in enumerate(sizes if dtype != torch.uint8 else []):
        x = gpu_fill(eng, n + (1 if i == 2 else 0), d, seed=80 + i, dtype=dtype)
        if i == 2:  # a view 1 row + 4 bytes in: not 16-B aligned
            flat = x.view(-1)[1 : 1 + n * d] if dtype == torch.float32 else x.view(-1)[2 : 2 + n * d]
            x = flat.view(n, d)
            assert x.data_ptr() % 16 != 0
        xs.append(x.float().cpu().numpy())
        shards.append(Shard(x, base))
        base += n + 1000 * (i + 1)  # gaps between the sources' global rows
    q = torch.from_numpy(O.fill_normal(1, d, seed=90))
    m = _lib.METRICS[metric]
    for k in (10, 100, 1000, 1024):
        assert eng._one_merge(shards, 1, k, m, None)
        one = eng.search(shards, q, m, k)
        Engine.ONE_MERGE = False
        try:
            per = eng.search(shards, q, m, k)
        finally:
            Engine.ONE_MERGE = True
        torch.cuda.synchronize()
        np.testing.assert_array_equal(one[1].cpu().numpy(), per[1].cpu().numpy())
        np.testing.assert_array_equal(one[0].cpu().numpy().view(np.uint32),
                                      per[0].cpu().numpy().view(np.uint32))
    # the rows against the float64 oracle over the concatenated sources
    allx = np.concatenate(xs)
    glob = np.concatenate([s.row_base + np.arange(s.n) for s in shards])
    od, orow = O.knn(allx, q.numpy(), metric, 100)
    gd, gr = eng.search(shards, q, m, 100)
    # (global rows increase with the concatenated index: the same tie order)
    check_topk(gd.cpu().numpy(), gr.cpu().numpy(), od, glob[orow], allx, q.numpy(), metric)


@pytest.mark.parametrize("metric", METRICS)
@pytest.mark.parametrize("dtype,n,d,nq,k", [
    (torch.float16, 400_000, 256, 1, 1000),   # one query, ~10^4-10^5 candidates
    (torch.float32, 300_000, 128, 3, 600),
    (torch.float16, 200_000, 1536, 5, 1000),  # configs[4]'s width
])
def test_int8_large_k_pruned_selects_bit_identical(eng, metric, dtype, n, d, nq, k):
    """k >= 512 through the int8 image (option i8_max_k raised): every
    select over the large candidate buffer first keeps the k smallest of each
    16 K slice in parallel (select_kernel MODE 3, knn_batch.hip) and then
    selects from those k-lists.  Results equal the exact scan bit for bit,
    and through the overflow fallback (force_fallback: the final select
    takes the fallback lists, never the pruned ones).  Reference: the
    select_k_unstable of index.py:165-168 with an unbounded maxval."""
    x = gpu_fill(eng, n, d, seed=71, dtype=dtype)
    q = O.fill_normal(nq, d, seed=72)
    q[0] = O.fill_normal(n, d, 71)[n // 3] if nq > 1 else q[0]  # a query near the corpus
    m = _lib.METRICS[metric]
    eng.clear_images()
    with _lib.options(i8_max_k=1024, batch_min_queries=1):
        assert _lib.filter_image_used(n, d, eng_dtype(dtype), nq, k, m)
        fd, fr = gpu_search(eng, x, q, metric, k)
        shard = Shard(x, 0)
        st = eng.scan(shard, torch.as_tensor(q).to(eng.device), m, k)
        counts, cap = eng.filter_counts(shard, nq, m, k, st)
        with _lib.options(force_fallback=1):
            gd, gr = gpu_search(eng, x, q, metric, k)
    with _lib.options(batched=0):
        sd, sr = gpu_search(eng, x, q, metric, k)
    eng.clear_images()
    assert cap > 2 * 16384  # the prune plan (select_prune_lists)
    print(f"candidate counts {counts.tolist()} cap {cap}")
    for dd, rr in ((fd, fr), (gd, gr)):
        np.testing.assert_array_equal(rr, sr)
        np.testing.assert_array_equal(dd.view(np.uint32), sd.view(np.uint32))


def eng_dtype(dtype):
    return _lib.DTYPE_F16 if dtype == torch.float16 else _lib.DTYPE_F32


@pytest.mark.parametrize("metric", METRICS)
def test_int8_k1000_default_masked_extreme_clustered(eng, metric):
    """k = 1 000 through the int8 image with the DEFAULT options (i8_max_k
    1 024 since round 6; batch_min_queries = 1 only sends the single query
    below the 4 GiB single-query rule): a mask, rows the image cannot
    represent, a clustered corpus and a query planted inside a cluster, each
    bit-identical to the exact scan, and the clean single query's ids
    against the float64 oracle.  Reference: index.py:161-168 (filter, then
    select_k_unstable with maxval 1 000)."""
    n, d, k = 150_000, 128, 1000
    m = _lib.METRICS[metric]
    assert _lib.get_option("i8_max_k") >= k
    cases = []
    xh = _extreme_rows(n, d, 81)
    mask = np.random.RandomState(82).rand(n) < 0.7
    cases.append(("extreme+mask", torch.from_numpy(xh).to(eng.device), mask,
                  O.fill_normal(1, d, seed=83)))
    xc = gpu_fill(eng, n, d, seed=84, cluster=1000)
    qc = O.fill_normal(n, d, 84, cluster=1000)[n // 2 : n // 2 + 1] + 0.01
    cases.append(("clustered, query in a cluster", xc, None, qc))
    xn = gpu_fill(eng, n, d, seed=85)
    qn = O.fill_normal(1, d, seed=86)
    cases.append(("clean", xn, None, qn))
    for name, x, mk, q in cases:
        eng.clear_images()
        with _lib.options(batch_min_queries=1):
            assert _lib.filter_image_used(n, d, _lib.DTYPE_F32, 1, k, m)
            fd, fr = gpu_search(eng, x, q, metric, k, mask=mk)
            assert id(x) in eng._images, name  # the int8 image served it
        with _lib.options(batched=0):
            sd, sr = gpu_search(eng, x, q, metric, k, mask=mk)
        np.testing.assert_array_equal(fr, sr, err_msg=name)
        np.testing.assert_array_equal(fd.view(np.uint32), sd.view(np.uint32), err_msg=name)
        if mk is not None:
            assert np.all(mk[fr[fr >= 0]]), name
    od, orow = O.knn(O.fill_normal(n, d, 85), qn, metric, k)
    check_topk(fd, fr, od, orow, O.fill_normal(n, d, 85), qn, metric)
    eng.clear_images()
