"""CPU oracle for fenix's brute-force kNN path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module; the product path (``fenix_amd``) never does and
fails loudly without its HIP library.

It restates (paths relative to the reference checkout, nrlugg/fenix):

* ``src/fenix/io/coder/coder.py:38-50`` — the metric formulas
  (:func:`distance_f64`, :func:`fenix_distance`);
* ``src/fenix/io/index/index.py:161-170`` — filter, distance column, top-k by
  ``select_k_unstable`` ascending (NaN after numbers), here with the
  deterministic ``(distance, row)`` tie-break (:func:`knn_numpy`, :func:`knn`);
* ``tests/test_flight.py:17-35`` — the clustered test corpus
  (:func:`fill_normal` with ``cluster``).

Pinning: ``tests/golden/`` holds outputs of the reference itself
(``tests/golden/make_golden.py`` imported fenix in the build container and ran
``io.index.call`` / ``Flight.search``); ``tests/test_oracle_golden.py`` checks
this restatement against them.
"""

from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libknnref.so")

METRIC_IDS = {"l2": 0, "euclidean": 0, "inner_product": 1, "dot": 1, "cosine": 2}

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_SCALE = np.float32(2.6428998e-05)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    z = z + _GOLDEN
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def _irwin_hall4(h: np.ndarray) -> np.ndarray:
    m = np.uint64(0xFFFF)
    s = (
        (h & m).astype(np.int64)
        + ((h >> np.uint64(16)) & m).astype(np.int64)
        + ((h >> np.uint64(32)) & m).astype(np.int64)
        + (h >> np.uint64(48)).astype(np.int64)
        - 131070
    )
    return s.astype(np.float32) * _SCALE


def fill_normal(
    n: int, d: int, seed: int, row_base: int = 0, cluster: int = 0, dtype=np.float32
) -> np.ndarray:
    """Portable corpus generator; bit-identical to ``fx_fill_normal`` (HIP)."""
    with np.errstate(over="ignore"):
        smix = np.uint64(seed) * _GOLDEN
        g = np.arange(row_base, row_base + n, dtype=np.uint64)[:, None]
        c = np.arange(d, dtype=np.uint64)[None, :]
        x = _irwin_hall4(_splitmix64(smix + g * np.uint64(d) + c))
        if cluster > 0:
            b0 = g // np.uint64(cluster) * np.uint64(cluster)
            x0 = _irwin_hall4(_splitmix64(smix + b0 * np.uint64(d) + c))
            x = x + np.float32(10.0) * x0
    return x.astype(dtype)


def distance_f64(x: np.ndarray, q: np.ndarray, metric: str) -> np.ndarray:
    """coder.py:38-50 in float64 with direct differences: [nq, n]."""
    x64 = np.asarray(x, dtype=np.float64)
    q64 = np.atleast_2d(np.asarray(q, dtype=np.float64))
    m = METRIC_IDS[metric]
    if m == 0:
        out = np.empty((q64.shape[0], x64.shape[0]))
        for i, qv in enumerate(q64):
            out[i] = np.sqrt(((x64 - qv) ** 2).sum(axis=1))
        return out
    dot = q64 @ x64.T
    if m == 1:
        return -dot
    nx = np.maximum(np.sqrt((x64 * x64).sum(axis=1)), 1e-12)
    nq = np.maximum(np.sqrt((q64 * q64).sum(axis=1)), 1e-12)
    return 0.5 - 0.5 * dot / (nq[:, None] * nx[None, :])


def topk_rows(dist: np.ndarray, k: int, row_base: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """Deterministic (distance asc, row asc) top-k per query; NaN after numbers."""
    dist = np.atleast_2d(dist)
    nq, n = dist.shape
    out_d = np.full((nq, k), np.nan)
    out_r = np.full((nq, k), -1, dtype=np.int64)
    rows = np.arange(n, dtype=np.int64) + row_base
    for i in range(nq):
        dv = dist[i]
        nan = np.isnan(dv)
        key = np.where(nan, np.inf, dv)
        order = np.lexsort((rows, nan, key))  # primary key, then NaN flag, then row
        take = order[:k]
        out_d[i, : take.size] = dv[take]
        out_r[i, : take.size] = rows[take]
    return out_d, out_r


def knn_numpy(
    x: np.ndarray,
    q: np.ndarray,
    metric: str,
    k: int,
    mask: Optional[np.ndarray] = None,
    row_base: int = 0,
) -> Tuple[np.ndarray, np.ndarray]:
    """Pure-numpy float64 restatement (small cases)."""
    d = distance_f64(x, q, metric)
    if mask is not None:
        keep = np.asarray(mask, dtype=bool)
        idx = np.nonzero(keep)[0]
        dsub = d[:, idx]
        od, orow = topk_rows(dsub, k)
        mapped = np.where(orow >= 0, idx[np.clip(orow, 0, None)] + row_base, -1)
        return od, mapped
    return topk_rows(d, k, row_base)


def fenix_distance(u: np.ndarray, v: np.ndarray, metric: str) -> np.ndarray:
    """coder.py:38-50 exactly as fenix evaluates it (torch CPU, f32)."""
    import torch
    import torch.nn.functional as F

    tu = torch.from_numpy(np.atleast_2d(np.asarray(u, dtype=np.float32)))
    tv = torch.from_numpy(np.asarray(v, dtype=np.float32))
    if metric in {"euclidean", "l2"}:
        return torch.cdist(tu, tv).numpy()
    if metric in {"cosine"}:
        tu = F.normalize(tu, dim=-1)
        tv = F.normalize(tv, dim=-1)
        return (0.5 - 0.5 * tu @ tv.transpose(-1, -2)).numpy()
    if metric in {"dot", "inner_product"}:
        return (-tu @ tv.transpose(-1, -2)).numpy()
    raise ValueError()


# ------------------------------------------------------------------ C library

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        i64, u64, vp = ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p
        L.fx_ref_fill.argtypes = [vp, i64, i64, u64, i64, i64]
        L.fx_ref_fill.restype = None
        L.fx_ref_knn.argtypes = [vp, ctypes.c_int, i64, i64, i64, vp, i64, ctypes.c_int, i64, vp,
                                 ctypes.c_int, ctypes.c_int, vp, vp]
        L.fx_ref_knn.restype = ctypes.c_int
        L.fx_ref_distances.argtypes = [vp, ctypes.c_int, i64, i64, vp, i64, ctypes.c_int,
                                       ctypes.c_int, vp]
        L.fx_ref_distances.restype = ctypes.c_int
        L.fx_ref_knn_gen.argtypes = [u64, i64, i64, i64, i64, ctypes.c_int, vp, vp, i64, vp, i64,
                                     ctypes.c_int, i64, ctypes.c_int, ctypes.c_int, vp, vp]
        L.fx_ref_knn_gen.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def fill_normal_c(n: int, d: int, seed: int, row_base: int = 0, cluster: int = 0) -> np.ndarray:
    x = np.empty((n, d), dtype=np.float32)
    lib().fx_ref_fill(_ptr(x), n, d, seed, row_base, cluster)
    return x


def bitmap(mask: np.ndarray) -> np.ndarray:
    """bool[n] -> uint32 bitmap (bit r of word r>>5), the C ABI mask format."""
    mask = np.asarray(mask, dtype=bool).ravel()
    words = (mask.size + 31) // 32
    padded = np.zeros(words * 32, dtype=bool)
    padded[: mask.size] = mask
    return np.packbits(padded, bitorder="little").view("<u4").astype(np.uint32)


def knn(
    x: np.ndarray,
    q: np.ndarray,
    metric: str,
    k: int,
    mask: Optional[np.ndarray] = None,
    row_base: int = 0,
    precision: int = 64,
    threads: int = 0,
) -> Tuple[np.ndarray, np.ndarray]:
    """C restatement (OpenMP).  x: f32 or f16 [n, d]; q: [nq, d]."""
    x = np.ascontiguousarray(x)
    if x.dtype == np.float32:
        dt = 0
    elif x.dtype == np.float16:
        dt = 1
        x = x.view(np.uint16)
    else:
        raise TypeError(x.dtype)
    q = np.ascontiguousarray(np.atleast_2d(q), dtype=np.float32)
    n, d = x.shape
    nq = q.shape[0]
    bm = None if mask is None else bitmap(mask)
    od = np.empty((nq, k), dtype=np.float64)
    orow = np.empty((nq, k), dtype=np.int64)
    rc = lib().fx_ref_knn(_ptr(x), dt, n, d, row_base, _ptr(q), nq, METRIC_IDS[metric], k,
                          _ptr(bm), precision, threads, _ptr(od), _ptr(orow))
    if rc != 0:
        raise ValueError("fx_ref_knn failed")
    return od, orow


def knn_gen(
    n: int,
    d: int,
    seed: int,
    q: np.ndarray,
    metric: str,
    k: int,
    row_base: int = 0,
    cluster: int = 0,
    dtype=np.float32,
    overrides: Optional[dict] = None,
    precision: int = 64,
    threads: int = 0,
) -> Tuple[np.ndarray, np.ndarray]:
    """:func:`knn` over ``fill_normal(n, d, seed, row_base, cluster, dtype)``
    generated block by block in C (never materialised: the full-size
    configs[3]/[4] corpora are 246 / 154 GB).  ``overrides``: {local row:
    [d] values} replacing generated rows (planted neighbours), cast to
    ``dtype`` like the generated ones."""
    q = np.ascontiguousarray(np.atleast_2d(q), dtype=np.float32)
    items = sorted((overrides or {}).items())
    rows = np.array([r for r, _ in items], dtype=np.int64)
    vals = np.ascontiguousarray(np.array([np.asarray(v, dtype=np.float32) for _, v in items],
                                         dtype=np.float32).reshape(len(items), d))
    nq = q.shape[0]
    od = np.empty((nq, k), dtype=np.float64)
    orow = np.empty((nq, k), dtype=np.int64)
    rc = lib().fx_ref_knn_gen(seed, row_base, n, d, cluster, int(np.dtype(dtype) == np.float16),
                              _ptr(rows), _ptr(vals), len(items), _ptr(q), nq,
                              METRIC_IDS[metric], k, precision, threads, _ptr(od), _ptr(orow))
    if rc != 0:
        raise ValueError("fx_ref_knn_gen failed")
    return od, orow


def distances(x: np.ndarray, q: np.ndarray, metric: str, precision: int = 64) -> np.ndarray:
    x = np.ascontiguousarray(x)
    dt = 0 if x.dtype == np.float32 else 1
    if dt == 1:
        x = x.view(np.uint16)
    q = np.ascontiguousarray(np.atleast_2d(q), dtype=np.float32)
    out = np.empty((q.shape[0], x.shape[0]), dtype=np.float64)
    rc = lib().fx_ref_distances(_ptr(x), dt, x.shape[0], x.shape[1], _ptr(q), q.shape[0],
                                METRIC_IDS[metric], precision, _ptr(out))
    if rc != 0:
        raise ValueError("fx_ref_distances failed")
    return out


def dequantize(codes: np.ndarray, scale: float, shift: int) -> np.ndarray:
    """quint8 codes -> float32 values exactly as QUInt8NDArray.dequantize
    (src/fenix/ex/arrow/quint8/quint8.py:53-54): float32(scale) * (codes - shift)."""
    return np.float32(scale) * (np.asarray(codes, dtype=np.float32) - np.float32(shift))
