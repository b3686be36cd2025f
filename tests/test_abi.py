"""The C-ABI library loads and exports exactly what include/fenix_knn.h
declares; argument validation runs without a GPU (no compute calls here)."""

from __future__ import annotations

import ctypes
import os
import re

import pytest

from fenix_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fenix_knn.h")


def declared_symbols():
    text = open(HEADER).read()
    return set(re.findall(r"^\s*(?:int|int64_t|uint64_t|const char\*)\s+(fx_\w+)\s*\(", text, re.M))


def test_header_and_binding_agree():
    assert declared_symbols() == set(_lib.SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for sym in declared_symbols():
        assert getattr(lib, sym) is not None
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for sym in declared_symbols():
        assert hasattr(raw, sym)


def test_library_is_gfx950():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_and_limits():
    lib = _lib.load()
    # 1.4: int8 images in permuted row order (1.3: int8 filter images; 1.2:
    # options, device-gated fallback)
    assert lib.fx_version() == 104
    assert _lib.max_k() == 1024


def test_options_round_trip_and_unknown_names():
    for name in _lib.OPTIONS:
        old = _lib.get_option(name)
        with _lib.options(**{name: old + 3}):
            assert _lib.get_option(name) == old + 3
        assert _lib.get_option(name) == old
    assert _lib.get_option("batched") == 1 and _lib.get_option("batch_min_queries") == 2
    with pytest.raises(ValueError, match="unknown option"):
        _lib.set_option("no_such_option", 1)


def test_product_library_reads_no_environment_switches():
    """Kernel selection is not reachable through the environment: the
    rejected variants and tuning knobs exist only in `make diag` builds.
    (rocPRIM, linked for the radix sorts, reads its own debug variables.)"""
    data = open(_lib.LIB_PATH, "rb").read()
    for name in (b"FX_BATCH", b"FX_FILTER_RING", b"FX_IMAGE_TILED", b"FX_FILTER_DIAG",
                 b"FX_SCAN_INTERLEAVE", b"FX_SCAN_PIPE", b"FX_SCAN_BLOCKS_PER_CU",
                 b"FX_MERGE_GROUP", b"FX_Q8_DMA"):
        assert name not in data, name
    assert _lib.host_sync_count() == 0


def test_invalid_arguments_are_rejected_before_any_device_work():
    with pytest.raises(ValueError, match="invalid shape"):
        _lib.knn_workspace_bytes(0, 8, _lib.DTYPE_F32, 1, 10)
    with pytest.raises(ValueError, match="dtype"):
        _lib.knn_workspace_bytes(10, 8, 7, 1, 10)
    with pytest.raises(NotImplementedError, match="k="):
        _lib.knn_workspace_bytes(10, 8, _lib.DTYPE_F32, 1, 1 << 31)
    with pytest.raises(ValueError):
        _lib.merge_workspace_bytes(1, 2, 10, 0)
    lib = _lib.load()
    rc = lib.fx_knn_search(None, 0, 10, 8, 0, None, 1, 0, 5, None, None, 0, None, None, None)
    assert rc == -1 and b"null" in lib.fx_last_error()
    rc = lib.fx_knn_distances(None, 0, 10, 8, None, 1, 9, None, None, None)
    assert rc == -1 and b"metric" in lib.fx_last_error()
    rc = lib.fx_fill_normal(None, 0, 10, 8, 0, 0, 0, None)
    assert rc == -1


def test_merge_workspace_needs_no_device():
    assert _lib.merge_workspace_bytes(4, 8, 100, 100) >= 4 * 8 * 100 * 8


def test_error_mapping():
    with pytest.raises(ValueError):
        _lib.check(-1)
    with pytest.raises(NotImplementedError):
        _lib.check(-2)
    with pytest.raises(_lib.FenixHipError):
        _lib.check(-3)
    _lib.check(0)


def test_metric_aliases_follow_coder():
    # coder.py:39 euclidean == l2, coder.py:47 dot == inner_product
    assert _lib.METRICS["euclidean"] == _lib.METRICS["l2"] == _lib.METRIC_L2
    assert _lib.METRICS["dot"] == _lib.METRICS["inner_product"] == _lib.METRIC_IP
    assert _lib.METRICS["cosine"] == _lib.METRIC_COS


def test_comm_argument_checks_without_gpu():
    """fx_comm_init_all rejects a device listed twice (one RCCL rank per
    device) and an empty list before touching RCCL or the GPU."""
    import ctypes

    from fenix_amd import _lib

    L = _lib.load()
    h = ctypes.c_void_p()
    two = (ctypes.c_int * 2)(0, 0)
    assert L.fx_comm_init_all(2, two, ctypes.byref(h)) == -1
    assert b"twice" in L.fx_last_error()
    assert L.fx_comm_init_all(0, two, ctypes.byref(h)) == -1
    assert L.fx_comm_destroy(None) == 0


def test_image8_row_permutation_is_a_bijection():
    """fx_filter_image8_perm: image row i holds corpus row (mult * i) % n, a
    bijection for every n (mult coprime with n), spreading consecutive corpus
    rows: the filter's samples are prefixes of the image, and a prefix of
    1/8 of its rows holds ~1/8 of every 1 000-row cluster."""
    import math

    import numpy as np

    for n in (0, 1, 2, 3, 7, 256, 1000, 65_537, 400_000, 1_000_003, 6_250_000):
        a = _lib.image8_perm(n)
        if n <= 2:
            assert a == 1
            continue
        assert math.gcd(a, n) == 1 and 0 < a < n
        if n <= 1_000_003:
            rows = (a * np.arange(n, dtype=np.uint64)) % np.uint64(n)
            assert len(np.unique(rows)) == n
    n = 1_000_003
    a = _lib.image8_perm(n)
    i = np.arange(n, dtype=np.int64)
    for frac in (8, 64):
        sample = ((a * i) % n)[: n // frac]
        per_cluster = np.bincount(sample // 1000, minlength=n // 1000 + 1)[:-1]
        expect = 1000 / frac
        assert per_cluster.min() >= 0.8 * expect - 1 and per_cluster.max() <= 1.2 * expect + 1
    with pytest.raises(ValueError):
        _lib.check(_lib.load().fx_filter_image8_perm(-1, ctypes.byref(ctypes.c_uint64())))
