"""ctypes binding of the gfx950 C ABI (``include/fenix_knn.h``).

The shared library is built in-tree by ``__graft_entry__.build()``
(``make -C fenix_amd/csrc`` -> ``fenix_amd/lib/libfenix_knn.so``).  There is no
CPU fallback: if the library or a GPU is missing, every search raises.
Error mapping mirrors the reference's surface: bad arguments -> ``ValueError``
(coder.py:50 raises ``ValueError()`` for an unknown metric), unsupported
shapes -> ``NotImplementedError``, HIP failures -> ``RuntimeError``.
"""

from __future__ import annotations

import contextlib
import ctypes
import hashlib
import os
import threading
from typing import Iterator

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FENIX_AMD_LIB") or os.path.join(HERE, "lib", "libfenix_knn.so")
# (FENIX_AMD_LIB: load a variant build instead, for tools/ A/B runs only)

DTYPE_F32 = 0
DTYPE_F16 = 1
DTYPE_QU8 = 2  # quint8 codes (fx_knn_*_ex entry points)
METRIC_L2 = 0
METRIC_IP = 1
METRIC_COS = 2

# coder.py:38-50: the metric names fenix accepts and their aliases
METRICS = {
    "l2": METRIC_L2,
    "euclidean": METRIC_L2,
    "inner_product": METRIC_IP,
    "dot": METRIC_IP,
    "cosine": METRIC_COS,
}

# every symbol include/fenix_knn.h declares
SYMBOLS = (
    "fx_version",
    "fx_last_error",
    "fx_device_count",
    "fx_max_k",
    "fx_knn_workspace_bytes",
    "fx_knn_workspace_bytes_img8",
    "fx_knn_search",
    "fx_knn_scan",
    "fx_knn_reduce",
    "fx_filter_image_bytes",
    "fx_filter_image",
    "fx_filter_image_used",
    "fx_knn_scan_img",
    "fx_knn_search_img",
    "fx_filter_image8_bytes",
    "fx_filter_image8",
    "fx_knn_scan_img8",
    "fx_knn_search_img8",
    "fx_knn_reduce_img8",
    "fx_filter_image8_typed",
    "fx_filter_image8_perm",
    "fx_knn_filter_counts",
    "fx_knn_filter_state",
    "fx_knn_distances",
    "fx_topk_merge_workspace_bytes",
    "fx_topk_merge",
    "fx_fill_normal",
    "fx_row_sqnorms",
    "fx_code_assign_workspace_bytes",
    "fx_code_assign",
    "fx_kmeans_step_workspace_bytes",
    "fx_kmeans_step",
    "fx_code_probe_workspace_bytes",
    "fx_code_probe",
    "fx_code_mask",
    "fx_knn_search_rows_workspace_bytes",
    "fx_knn_search_rows",
    "fx_mask_compact_workspace_bytes",
    "fx_mask_compact",
    "fx_knn_search_ex_workspace_bytes",
    "fx_knn_search_ex",
    "fx_knn_search_shards_workspace_bytes",
    "fx_knn_search_shards",
    "fx_knn_distances_ex",
    "fx_comm_init_all",
    "fx_comm_destroy",
    "fx_allgather_topk",
    "fx_set_option",
    "fx_get_option",
    "fx_host_sync_count",
)

# process options of the library (fx_set_option, include/fenix_knn.h): the
# "batched", "batch_min_queries" and "filter_image" are user switches, the rest
# test switches
OPTIONS = ("batched", "batch_min_queries", "batch_cap", "batch_sample_ratio", "force_fallback",
           "scan_interleave", "q8_dma", "filter_image", "batch_ub_test", "single_query_image",
           "i8_max_k", "img6", "img8", "i8_sample_ratio", "i8_grow_ratio", "select_prune")

_lock = threading.Lock()
_lib = None


class Corpus(ctypes.Structure):
    """struct fx_corpus (include/fenix_knn.h)."""

    _fields_ = [
        ("data", ctypes.c_void_p),
        ("dtype", ctypes.c_int),
        ("n", ctypes.c_int64),
        ("d", ctypes.c_int64),
        ("row_base", ctypes.c_int64),
        ("scale", ctypes.c_float),
        ("zero_point", ctypes.c_int32),
    ]


class FenixHipError(RuntimeError):
    """A HIP runtime failure inside the kNN engine."""


def load() -> ctypes.CDLL:
    """Load (once) and type the shared library; raise loudly if it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"fenix_amd HIP library not built: {LIB_PATH} is missing "
                "(run __graft_entry__.build() or `make -C fenix_amd/csrc`)"
            )
        L = ctypes.CDLL(LIB_PATH)
        i64, sz, vp, ci = ctypes.c_int64, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int
        L.fx_version.argtypes = []
        L.fx_version.restype = ci
        L.fx_last_error.argtypes = []
        L.fx_last_error.restype = ctypes.c_char_p
        L.fx_device_count.argtypes = [ctypes.POINTER(ci)]
        L.fx_device_count.restype = ci
        L.fx_max_k.argtypes = []
        L.fx_max_k.restype = i64
        L.fx_knn_workspace_bytes.argtypes = [i64, i64, ci, i64, i64, ctypes.POINTER(sz)]
        L.fx_knn_workspace_bytes.restype = ci
        L.fx_knn_workspace_bytes_img8.argtypes = [i64, i64, ci, i64, i64, ci, ctypes.POINTER(sz)]
        L.fx_knn_workspace_bytes_img8.restype = ci
        L.fx_knn_search.argtypes = [vp, ci, i64, i64, i64, vp, i64, ci, i64, vp, vp, sz, vp, vp,
                                    vp]
        L.fx_knn_search.restype = ci
        L.fx_knn_scan.argtypes = [vp, ci, i64, i64, i64, vp, i64, ci, i64, vp, vp, sz, vp]
        L.fx_knn_scan.restype = ci
        L.fx_knn_reduce.argtypes = [vp, ci, i64, i64, i64, vp, i64, ci, i64, vp, vp, sz, vp, vp,
                                    vp]
        L.fx_knn_reduce.restype = ci
        L.fx_filter_image_bytes.argtypes = [i64, i64, ctypes.POINTER(sz), ctypes.POINTER(sz)]
        L.fx_filter_image_bytes.restype = ci
        L.fx_filter_image.argtypes = [vp, i64, i64, vp, vp, vp]
        L.fx_filter_image.restype = ci
        L.fx_filter_image_used.argtypes = [i64, i64, ci, i64, i64, ci, ctypes.POINTER(ci)]
        L.fx_filter_image_used.restype = ci
        L.fx_knn_scan_img.argtypes = [vp, ci, i64, i64, i64, vp, vp, vp, i64, ci, i64, vp, vp, sz,
                                      vp]
        L.fx_knn_scan_img.restype = ci
        L.fx_knn_search_img.argtypes = [vp, ci, i64, i64, i64, vp, vp, vp, i64, ci, i64, vp, vp,
                                        sz, vp, vp, vp]
        L.fx_knn_search_img.restype = ci
        L.fx_filter_image8_bytes.argtypes = [i64, i64, ctypes.POINTER(sz), ctypes.POINTER(sz)]
        L.fx_filter_image8_bytes.restype = ci
        L.fx_filter_image8.argtypes = [vp, i64, i64, vp, vp, vp]
        L.fx_filter_image8.restype = ci
        L.fx_filter_image8_typed.argtypes = [vp, ci, i64, i64, vp, vp, vp]
        L.fx_filter_image8_typed.restype = ci
        L.fx_filter_image8_perm.argtypes = [i64, ctypes.POINTER(ctypes.c_uint64)]
        L.fx_filter_image8_perm.restype = ci
        L.fx_knn_filter_counts.argtypes = [vp, ci, i64, i64, i64, ci, i64, ci, vp, sz, vp,
                                           ctypes.POINTER(i64), vp]
        L.fx_knn_filter_counts.restype = ci
        L.fx_knn_filter_state.argtypes = [vp, ci, i64, i64, i64, ci, i64, ci, vp, sz, vp, vp, vp,
                                          vp]
        L.fx_knn_filter_state.restype = ci
        L.fx_knn_scan_img8.argtypes = L.fx_knn_scan_img.argtypes
        L.fx_knn_scan_img8.restype = ci
        L.fx_knn_search_img8.argtypes = L.fx_knn_search_img.argtypes
        L.fx_knn_search_img8.restype = ci
        L.fx_knn_reduce_img8.argtypes = [vp, ci, i64, i64, i64, vp, vp, i64, ci, i64, vp, vp, sz,
                                         vp, vp, vp]
        L.fx_knn_reduce_img8.restype = ci
        L.fx_knn_distances.argtypes = [vp, ci, i64, i64, vp, i64, ci, vp, vp, vp]
        L.fx_knn_distances.restype = ci
        L.fx_topk_merge_workspace_bytes.argtypes = [i64, i64, i64, i64, ctypes.POINTER(sz)]
        L.fx_topk_merge_workspace_bytes.restype = ci
        L.fx_topk_merge.argtypes = [vp, vp, i64, i64, i64, i64, vp, sz, vp, vp, vp]
        L.fx_topk_merge.restype = ci
        L.fx_fill_normal.argtypes = [vp, ci, i64, i64, ctypes.c_uint64, i64, i64, vp]
        L.fx_fill_normal.restype = ci
        L.fx_row_sqnorms.argtypes = [vp, ci, i64, i64, vp, vp]
        L.fx_row_sqnorms.restype = ci
        psz = ctypes.POINTER(sz)
        L.fx_code_assign_workspace_bytes.argtypes = [i64, i64, i64, i64, psz]
        L.fx_code_assign_workspace_bytes.restype = ci
        L.fx_code_assign.argtypes = [vp, ci, i64, i64, vp, i64, i64, ci, vp, sz, vp, vp, vp, vp]
        L.fx_code_assign.restype = ci
        L.fx_kmeans_step_workspace_bytes.argtypes = [i64, i64, i64, i64, psz]
        L.fx_kmeans_step_workspace_bytes.restype = ci
        L.fx_kmeans_step.argtypes = [vp, ci, i64, i64, i64, vp, i64, ci, vp, sz, vp]
        L.fx_kmeans_step.restype = ci
        L.fx_code_probe_workspace_bytes.argtypes = [i64, i64, i64, psz]
        L.fx_code_probe_workspace_bytes.restype = ci
        L.fx_code_probe.argtypes = [vp, i64, i64, i64, i64, vp, sz, vp, vp, vp, vp]
        L.fx_code_probe.restype = ci
        L.fx_code_mask.argtypes = [vp, i64, vp, i64, vp, vp, vp, vp]
        L.fx_code_mask.restype = ci
        L.fx_knn_search_rows_workspace_bytes.argtypes = [i64, i64, ci, i64, i64, psz]
        L.fx_knn_search_rows_workspace_bytes.restype = ci
        L.fx_knn_search_rows.argtypes = [vp, ci, i64, i64, i64, vp, i64, vp, i64, ci, i64, vp, sz,
                                         vp, vp, vp]
        L.fx_knn_search_rows.restype = ci
        L.fx_mask_compact_workspace_bytes.argtypes = [i64, psz]
        L.fx_mask_compact_workspace_bytes.restype = ci
        L.fx_mask_compact.argtypes = [vp, i64, vp, sz, vp, vp, vp]
        L.fx_mask_compact.restype = ci
        pc_ = ctypes.POINTER(Corpus)
        L.fx_knn_search_ex_workspace_bytes.argtypes = [pc_, i64, i64, i64, psz]
        L.fx_knn_search_ex_workspace_bytes.restype = ci
        L.fx_knn_search_ex.argtypes = [pc_, vp, i64, vp, i64, ci, i64, vp, vp, sz, vp, vp, vp]
        L.fx_knn_search_ex.restype = ci
        L.fx_knn_search_shards_workspace_bytes.argtypes = [pc_, ci, i64, i64, psz]
        L.fx_knn_search_shards_workspace_bytes.restype = ci
        L.fx_knn_search_shards.argtypes = [pc_, ci, vp, i64, ci, i64, vp, vp, sz, vp, vp, vp]
        L.fx_knn_search_shards.restype = ci
        L.fx_knn_distances_ex.argtypes = [pc_, vp, i64, ci, vp, vp, vp]
        L.fx_knn_distances_ex.restype = ci
        L.fx_comm_init_all.argtypes = [ci, ctypes.POINTER(ci), ctypes.POINTER(vp)]
        L.fx_comm_init_all.restype = ci
        L.fx_comm_destroy.argtypes = [vp]
        L.fx_comm_destroy.restype = ci
        pvp = ctypes.POINTER(vp)
        L.fx_allgather_topk.argtypes = [vp, pvp, pvp, i64, i64, pvp, pvp, pvp]
        L.fx_allgather_topk.restype = ci
        L.fx_set_option.argtypes = [ctypes.c_char_p, i64]
        L.fx_set_option.restype = ci
        L.fx_get_option.argtypes = [ctypes.c_char_p, ctypes.POINTER(i64)]
        L.fx_get_option.restype = ci
        L.fx_host_sync_count.argtypes = []
        L.fx_host_sync_count.restype = ctypes.c_uint64
        _lib = L
        return L


def check(rc: int) -> None:
    if rc == 0:
        return
    msg = (load().fx_last_error() or b"").decode(errors="replace")
    if rc == -1:
        raise ValueError(msg)
    if rc == -2:
        raise NotImplementedError(msg)
    raise FenixHipError(msg)


def max_k() -> int:
    return int(load().fx_max_k())


# Per-shape planning answers (workspace sizes, whether a search reads a filter
# image) depend on the shape and the process options only: memoised, keyed on
# the options' generation (set_option bumps it), so a serving loop over many
# shards does not re-plan each search in Python-to-C calls.
_opt_gen = 0
_plan_cache: dict = {}
_PLAN_CACHE_MAX = 4096


def _planned(key: tuple, compute):
    hit = _plan_cache.get((_opt_gen, key))
    if hit is None:
        if len(_plan_cache) >= _PLAN_CACHE_MAX:
            _plan_cache.clear()
        hit = _plan_cache[(_opt_gen, key)] = compute()
    return hit


def knn_workspace_bytes(n: int, d: int, dtype: int, nq: int, k: int, img8: bool = True) -> int:
    """fx_knn_workspace_bytes_img8: workspace of a search of this shape that is
    (img8) or is not given an int8 filter image (4x the candidate buffers), on
    the current device (its CU count sizes the scan's lists: part of the key)."""
    def compute() -> int:
        out = ctypes.c_size_t(0)
        check(load().fx_knn_workspace_bytes_img8(n, d, dtype, nq, k, int(bool(img8)),
                                                 ctypes.byref(out)))
        return int(out.value)

    return _planned(("ws", _current_device(), n, d, dtype, nq, k, bool(img8)), compute)


def _current_device() -> int:
    import torch

    return torch.cuda.current_device() if torch.cuda.is_available() else -1


def filter_image_used(n: int, d: int, dtype: int, nq: int, k: int, metric: int) -> bool:
    """True when a search of this shape runs the batched filter over f32 rows,
    which then streams an fp16 filter image if one is given (fx_filter_image)."""
    def compute() -> bool:
        out = ctypes.c_int(0)
        check(load().fx_filter_image_used(n, d, dtype, nq, k, metric, ctypes.byref(out)))
        return bool(out.value)

    return _planned(("img", n, d, dtype, nq, k, metric), compute)


def image8_perm(n: int) -> int:
    """fx_filter_image8_perm: int8 image row i holds corpus row (mult * i) % n."""
    out = ctypes.c_uint64(0)
    check(load().fx_filter_image8_perm(n, ctypes.byref(out)))
    return int(out.value)


def merge_workspace_bytes(nq: int, parts: int, kin: int, k: int) -> int:
    out = ctypes.c_size_t(0)
    check(load().fx_topk_merge_workspace_bytes(nq, parts, kin, k, ctypes.byref(out)))
    return int(out.value)


def device_count() -> int:
    c = ctypes.c_int(0)
    check(load().fx_device_count(ctypes.byref(c)))
    return int(c.value)


def _ws(fn, *args) -> int:
    out = ctypes.c_size_t(0)
    check(fn(*args, ctypes.byref(out)))
    return int(out.value)


def code_assign_workspace_bytes(n: int, d: int, nb: int, ks: int) -> int:
    return _ws(load().fx_code_assign_workspace_bytes, n, d, nb, ks)


def kmeans_workspace_bytes(nb: int, bs: int, d: int, ks: int) -> int:
    return _ws(load().fx_kmeans_step_workspace_bytes, nb, bs, d, ks)


def code_probe_workspace_bytes(nq: int, nb: int, ks: int) -> int:
    return _ws(load().fx_code_probe_workspace_bytes, nq, nb, ks)


def search_rows_workspace_bytes(nrows: int, d: int, dtype: int, nq: int, k: int) -> int:
    return _ws(load().fx_knn_search_rows_workspace_bytes, nrows, d, dtype, nq, k)


def compact_workspace_bytes(n: int) -> int:
    return _ws(load().fx_mask_compact_workspace_bytes, n)


def search_ex_workspace_bytes(corpus: "Corpus", nrows: int, nq: int, k: int) -> int:
    out = ctypes.c_size_t(0)
    check(load().fx_knn_search_ex_workspace_bytes(ctypes.byref(corpus), nrows, nq, k,
                                                  ctypes.byref(out)))
    return int(out.value)


def search_shards_workspace_bytes(corpora, nq: int, k: int) -> int:
    """fx_knn_search_shards_workspace_bytes over a ctypes array of Corpus."""
    out = ctypes.c_size_t(0)
    check(load().fx_knn_search_shards_workspace_bytes(corpora, len(corpora), nq, k,
                                                      ctypes.byref(out)))
    return int(out.value)


def set_option(name: str, value: int) -> None:
    """fx_set_option: a process-wide library option (OPTIONS).  Options set
    through the C ABI directly bypass the planning memo: use this."""
    global _opt_gen
    check(load().fx_set_option(name.encode(), int(value)))
    _opt_gen += 1


def get_option(name: str) -> int:
    out = ctypes.c_int64(0)
    check(load().fx_get_option(name.encode(), ctypes.byref(out)))
    return int(out.value)


@contextlib.contextmanager
def options(**kw: int) -> Iterator[None]:
    """Set library options for the duration of a block (tests, tools)."""
    old = {k: get_option(k) for k in kw}
    try:
        for k, v in kw.items():
            set_option(k, v)
        yield
    finally:
        for k, v in old.items():
            set_option(k, v)


def host_sync_count() -> int:
    """fx_host_sync_count: host-blocking synchronisations inside the library."""
    return int(load().fx_host_sync_count())


_sha = None


def library_sha() -> str:
    """SHA-256 (first 16 hex digits) of the loaded shared library file: stamps
    profiles so a measurement is matched to the build it came from."""
    global _sha
    if _sha is None:
        h = hashlib.sha256()
        with open(LIB_PATH, "rb") as f:
            for blk in iter(lambda: f.read(1 << 20), b""):
                h.update(blk)
        _sha = h.hexdigest()[:16]
    return _sha


CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
BUILD_INFO = os.path.join(HERE, "lib", "build_info.json")


def sources_sha() -> str:
    """SHA-256 (16 hex digits) over the library's sources (csrc/*.hip, *.h,
    the Makefile and include/*.h, by name and content, sorted)."""
    h = hashlib.sha256()
    files = [os.path.join(CSRC, f) for f in os.listdir(CSRC)
             if f.endswith((".hip", ".h")) or f == "Makefile"]
    files += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    for p in sorted(files):
        h.update(os.path.relpath(p, os.path.dirname(HERE)).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def build_info() -> dict:
    """What ``__graft_entry__.build()`` recorded when it last ran make
    (``build_mode``: "make"; ``build_exercised``: whether make recompiled
    anything; the library and source hashes it produced), plus whether the
    library loaded now is that build and the sources on disk are its sources.
    Empty fields when no build() record exists (a library built by hand)."""
    import json

    rec = {}
    try:
        with open(BUILD_INFO) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        rec = {"build_mode": None, "build_exercised": None}
    rec["library_is_recorded_build"] = rec.get("library_sha") == library_sha()
    rec["sources_match"] = rec.get("sources_sha") == sources_sha()
    return rec
