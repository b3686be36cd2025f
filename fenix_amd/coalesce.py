"""Request coalescing for concurrent single-query searches (serving).

The reference serves every ``Flight.search`` as its own ``do_exchange`` call
(src/fenix/flight.py:62-77 -> io.index.call), and so does this engine: one
exact scan of the whole column per query.  On a large resident column that
scan is HBM-bound (10M x 768 f32: 4.4 ms), while a batch of queries costs
about one pass over the column through the fp16 filter (256 queries: 8.2 ms,
DESIGN.md §3.6).  So when requests arrive while the device is busy, they are
worth running together.

``Coalescer`` does that with no added latency at low load: the first request
for a key runs at once (it becomes the *leader*); requests arriving while the
leader's batch runs are queued, and when the batch finishes the first queued
request becomes the leader of the next batch (the whole queue).  Results are
exact and per request: the
batch runs with the largest k asked for and each request gets the prefix of
its own length (a top-K list sorted by (distance, row) starts with the top-k
for every k <= K).  An exception in a batch is raised in every request of it.

Only the plain case is coalesced (one query, no filter mask, no probe set);
``FENIX_AMD_COALESCE=0`` turns it off.  The module is torch-free so its
bookkeeping is tested on the CPU with a stand-in search function.
"""

from __future__ import annotations

import os
import threading
from typing import Any, Callable, Dict, Hashable, List, Optional, Tuple

import numpy as np

# run(queries [n, d] float32, K) -> (dist [n, K], rows [n, K], ...): every
# returned array is indexed [query, rank, ...] and sliced per request
RunFn = Callable[[np.ndarray, int], Tuple[np.ndarray, ...]]


def enabled() -> bool:
    return os.environ.get("FENIX_AMD_COALESCE", "1") != "0"


class _Request:
    __slots__ = ("query", "k", "wake", "promoted", "parts", "error")

    def __init__(self, query: np.ndarray, k: int) -> None:
        self.query = query
        self.k = k
        self.wake = threading.Event()  # result ready, or promoted to leader
        self.promoted = False
        self.parts: Optional[Tuple[np.ndarray, ...]] = None
        self.error: Optional[BaseException] = None


class Coalescer:
    """Groups concurrent ``search(key, run, query, k)`` calls with equal keys.

    ``run(queries [n, d] float32, K) -> (dist [n, K], rows [n, K], ...)``
    executes one batch (host arrays; any further arrays, such as the result
    rows' vectors [n, K, d], are sliced per request the same way).  A leader runs one batch — everything queued for
    its key, at most ``max_batch`` — then hands leadership to the first
    request still queued, so no caller serves other callers' batches after
    its own result is ready."""

    def __init__(self, max_batch: int = 1024) -> None:
        self.max_batch = max_batch
        self._lock = threading.Lock()
        self._queues: Dict[Hashable, List[_Request]] = {}
        self._running: set = set()
        self.batches = 0   # statistics (tests, tools/bench_flight.py)
        self.requests = 0

    def search(self, key: Hashable, run: RunFn, query: np.ndarray, k: int
               ) -> Tuple[np.ndarray, ...]:
        req = _Request(np.ascontiguousarray(query, dtype=np.float32).reshape(-1), int(k))
        with self._lock:
            self.requests += 1
            self._queues.setdefault(key, []).append(req)
            lead = key not in self._running
            if lead:
                self._running.add(key)
        if lead:
            self._lead_once(key, run)
        while True:
            req.wake.wait()
            if req.promoted and req.parts is None and req.error is None:
                req.promoted = False
                req.wake.clear()
                self._lead_once(key, run)
                continue
            break
        if req.error is not None:
            raise req.error
        return req.parts

    def _lead_once(self, key: Hashable, run: RunFn) -> None:
        with self._lock:
            queue = self._queues.get(key, [])
            batch, rest = queue[: self.max_batch], queue[self.max_batch :]
            self._queues[key] = rest
            self.batches += 1
        self._run(batch, run)
        with self._lock:
            rest = self._queues.get(key, [])
            if rest:
                rest[0].promoted = True
                rest[0].wake.set()
            else:
                self._queues.pop(key, None)
                self._running.discard(key)

    @staticmethod
    def _run(batch: List[_Request], run: RunFn) -> None:
        try:
            kmax = max(r.k for r in batch)
            parts = run(np.stack([r.query for r in batch]), kmax)
            for i, r in enumerate(batch):
                r.parts = tuple(p[i : i + 1, : r.k] for p in parts)
        except BaseException as e:  # every request of the batch sees the failure
            for r in batch:
                r.error = e
        finally:
            for r in batch:
                r.wake.set()


_DEFAULT: Optional[Coalescer] = None
_DLOCK = threading.Lock()


def default() -> Coalescer:
    global _DEFAULT
    with _DLOCK:
        if _DEFAULT is None:
            _DEFAULT = Coalescer()
        return _DEFAULT


def describe(c: Any) -> Dict[str, int]:
    return {"batches": c.batches, "requests": c.requests}
