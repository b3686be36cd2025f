"""Parity helpers shared by the GPU tests.

Parity rule (from BASELINE.json north_star):
* row ids: bit-exact against the float64 oracle under the (distance, row)
  tie-break.  The GPU computes in float32, so two rows whose float64
  distances are closer than the float32 resolution of the computation
  (``near``: 2e-6 relative to the distance for L2, to the magnitude of the
  summed terms for inner product / cosine) are a NEAR-TIE whose order
  float32 cannot decide; only those may differ.  With no
  near-tie in a case (the golden fixtures, most random cases) this is plain
  array equality, and the helper counts how many positions relied on it.
* distances: |gpu - f64| <= 1e-5 * max(|f64|, scale) where ``scale`` is the
  magnitude of the terms being summed (|q||x| for inner products, 1 for
  cosine, |q|+|x| for L2) — relative error on a cancelled sum is measured
  against what was summed, not against the tiny result.
"""

from __future__ import annotations

import numpy as np

DIST_RTOL = 1e-5
NEAR_RTOL = 2e-6


def scale_of(x: np.ndarray, q: np.ndarray, metric: str) -> np.ndarray:
    xn = float(np.sqrt((np.asarray(x, dtype=np.float64) ** 2).sum(axis=1)).max()) if len(x) else 0.0
    qn = np.sqrt((np.asarray(q, dtype=np.float64) ** 2).sum(axis=1))
    if metric in ("inner_product", "dot"):
        return np.maximum(qn * xn, 1e-30)
    if metric == "cosine":
        return np.ones_like(qn)
    return np.maximum(qn + xn, 1e-30)


def check_topk(gd, gr, od, orow, x, q, metric, allow_near_ties=True, details=None):
    """Return the number of near-tie positions used; raise AssertionError on a
    real mismatch.  ``details`` (a list): receives one dict per near-tie
    position (query, position, GPU row, oracle row, their float64 distances)."""
    gd = np.asarray(gd, dtype=np.float64)
    od = np.asarray(od, dtype=np.float64)
    gr = np.asarray(gr)
    orow = np.asarray(orow)
    assert gd.shape == od.shape and gr.shape == orow.shape
    sc = scale_of(x, q, metric)
    near_used = 0
    for i in range(gr.shape[0]):
        valid_o = orow[i] >= 0
        valid_g = gr[i] >= 0
        np.testing.assert_array_equal(valid_g, valid_o, err_msg=f"query {i}: filled slots differ")
        nv = int(valid_o.sum())
        g, o = gr[i, :nv], orow[i, :nv]
        assert len(np.unique(g)) == nv, f"query {i}: duplicate rows"
        tol_d = DIST_RTOL * np.fmax(np.abs(od[i, :nv]), sc[i])
        both_nan = np.isnan(gd[i, :nv]) & np.isnan(od[i, :nv])
        err = np.where(both_nan, 0.0, np.abs(gd[i, :nv] - od[i, :nv]))
        assert np.all(err <= tol_d), (
            f"query {i}: distance error {np.nanmax(err / np.maximum(tol_d, 1e-300))}x tolerance"
        )
        # GPU order is its own (distance, row) order
        for j in range(nv - 1):
            a, b = gd[i, j], gd[i, j + 1]
            if np.isnan(a):
                assert np.isnan(b) and g[j] < g[j + 1]
            elif not np.isnan(b):
                assert a < b or (a == b and g[j] < g[j + 1]), f"query {i}: not sorted at {j}"
        if np.array_equal(g, o):
            continue
        assert allow_near_ties, f"query {i}: ids differ at {np.nonzero(g != o)[0][:10]}"
        # float32 resolution of the computation: for L2 (direct differences)
        # relative to the distance; for dot-product metrics relative to the
        # magnitude of the summed terms (a cosine of 0.995 between large-norm
        # vectors carries ~1e-7 absolute error however small 0.5-0.5c is)
        if metric in ("l2", "euclidean"):
            near = NEAR_RTOL * float(np.nanmax(np.abs(od[i, :nv])))
        else:
            near = NEAR_RTOL * float(sc[i])
        pos_of = {int(r): j for j, r in enumerate(o)}
        for j in np.nonzero(g != o)[0]:
            r = int(g[j])
            if r in pos_of:
                jj = pos_of[r]
                assert abs(od[i, jj] - od[i, j]) <= near, (
                    f"query {i} pos {j}: row {r} belongs at {jj} "
                    f"(d64 {od[i, jj]!r} vs {od[i, j]!r})"
                )
                d64_gpu_row = float(od[i, jj])
            else:
                # boundary near-tie: row r must be as close as the last kept one
                assert abs(gd[i, j] - od[i, nv - 1]) <= near + DIST_RTOL * abs(od[i, nv - 1]), (
                    f"query {i} pos {j}: row {r} not in oracle top-k"
                )
                d64_gpu_row = None  # outside the oracle's top-k: its f64 distance is not at hand
            near_used += 1
            if details is not None:
                details.append({"query": i, "pos": int(j), "gpu_row": r, "oracle_row": int(o[j]),
                                "gpu_f32_dist": float(gd[i, j]), "gpu_row_d64": d64_gpu_row,
                                "oracle_row_d64": float(od[i, j]), "near_tol": near})
    return near_used
