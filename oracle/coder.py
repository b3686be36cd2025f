"""CPU restatement of fenix's coder (coded index) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module; nothing under fenix_amd/ imports it.  float64 numpy, following
src/fenix/io/coder/coder.py of nrlugg/fenix line by line:

* ``normalize``      F.normalize(x, dim=-1): x / max(||x||, 1e-12)  (coder.py:43-44)
* ``distance``       coder.py:38-50 (direct differences for l2 — cdist's matmul
                     expansion above 25 rows is a rounding artefact, not the metric)
* ``update``         one k-means step of one codebook (coder.py:53-65): argmin over
                     the codewords, torch.index_reduce(q, 0, i, v, "mean") with
                     include_self (the codeword counts as one sample of its mean)
* ``composite``      composite scores of coder.call (coder.py:171-181):
                     score[c] = sum_j d[j, digit_j(c)], c = sum_j digit_j ks^(nb-1-j)
* ``call``           coder.call (coder.py:143-194) with the deterministic
                     (score, code) order; maxval = 1 -> per-codebook argmin
* ``make``           coder.make's training loop (coder.py:94-118) driven by the
                     global ``np.random`` state exactly as the reference consumes it

Pinned by tests/golden/g5_coder.npz (outputs of the reference itself,
tests/golden/make_golden_coder.py): tests/test_oracle_coder.py.
"""

from __future__ import annotations

import numpy as np

from .oracle import METRIC_IDS

_KIND = {0: "l2", 1: "dot", 2: "cosine"}


def _kind(metric: str) -> str:
    return _KIND[METRIC_IDS[metric]]


def normalize(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.float64)
    n = np.sqrt((x * x).sum(-1, keepdims=True))
    return x / np.maximum(n, 1e-12)


def distance(u: np.ndarray, v: np.ndarray, metric: str) -> np.ndarray:
    """[rows(u), rows(v)] float64 distances (coder.py:38-50)."""
    m = _kind(metric)
    u = np.asarray(u, dtype=np.float64)
    v = np.asarray(v, dtype=np.float64)
    if m == "l2":
        out = np.empty((u.shape[0], v.shape[0]))
        step = max(1, (1 << 24) // max(1, v.size))
        for s in range(0, u.shape[0], step):
            diff = u[s : s + step, None, :] - v[None, :, :]
            out[s : s + step] = np.sqrt((diff * diff).sum(-1))
        return out
    if m == "cosine":
        return 0.5 - 0.5 * normalize(u) @ normalize(v).T
    return -(u @ v.T)


def update(q: np.ndarray, v: np.ndarray, metric: str) -> np.ndarray:
    """coder.py:53-65 for one codebook: q [ks, D], v [bs, D] -> new q."""
    q = np.asarray(q, dtype=np.float64)
    v = np.asarray(v, dtype=np.float64)
    cos = _kind(metric) == "cosine"
    if cos:
        q, v = normalize(q), normalize(v)
    i = np.argmin(distance(v, q, metric), axis=1)
    s = q.copy()
    c = np.ones(q.shape[0])
    np.add.at(s, i, v)
    np.add.at(c, i, 1.0)
    q = s / c[:, None]
    return normalize(q) if cos else q


def update_all(q: np.ndarray, v: np.ndarray, metric: str) -> np.ndarray:
    """torch.vmap(update) over codebooks: q [nb, ks, D], v [nb, bs, D]."""
    return np.stack([update(q[j], v[j], metric) for j in range(q.shape[0])])


def digits(nb: int, ks: int) -> np.ndarray:
    """[nb, ks^nb]: digit j of every composite code (coder.py:177)."""
    c = np.arange(ks**nb, dtype=np.int64)
    return np.stack([(c // ks ** (nb - 1 - j)) % ks for j in range(nb)])


def composite(d: np.ndarray, nb: int, ks: int) -> np.ndarray:
    """d [m, nb*ks] distances to the flattened codewords -> [m, ks^nb] scores."""
    d = d.reshape(-1, nb, ks)
    dg = digits(nb, ks)
    return sum(d[:, j, dg[j]] for j in range(nb))


def call(target: np.ndarray, tensor: np.ndarray, metric: str, maxval: int | None) -> np.ndarray:
    """coder.py:143-194 on numpy: [m, maxval] (or [m, ks^nb]) composite codes,
    ascending by (score, code)."""
    nb, ks, _ = tensor.shape
    d = distance(target, tensor.reshape(nb * ks, -1), metric)
    if maxval == 1:  # independent terms: the composite argmin is per codebook
        dd = d.reshape(-1, nb, ks)
        code = np.zeros(dd.shape[0], dtype=np.int64)
        for j in range(nb):
            code = code * ks + np.argmin(dd[:, j], axis=1)
        return code[:, None]
    s = composite(d, nb, ks)
    order = np.argsort(s, axis=1, kind="stable")
    return order if maxval is None else order[:, :maxval]


def make(x: np.ndarray, metric: str, codebook_size: int, num_codebooks: int, batch_size: int,
         num_epochs: int) -> np.ndarray:
    """coder.py:94-118 on numpy, consuming np.random like the reference:
    initial codewords = rows with permutation value < ks*nb (in row order), then
    per epoch a permutation cut into batches of nb*bs rows, each batch's rows in
    row order viewed as [nb, bs, D]."""
    n = x.shape[0]
    ks, nb, bs = codebook_size, num_codebooks, batch_size
    init = np.random.permutation(n) < ks * nb
    coding = np.asarray(x[init], dtype=np.float64).reshape(nb, ks, -1)
    for _ in range(num_epochs):
        step = nb * bs
        rows = np.random.permutation(n)
        rows = rows[: rows.size // step * step]
        for idx in np.array_split(rows, rows.size // step):
            sel = np.zeros(n, dtype=np.bool_)
            np.put(sel, idx, True)
            coding = update_all(coding, x[sel].reshape(nb, bs, -1), metric)
    return coding
