"""The generating oracle (oracle.knn_gen, fx_ref_knn_gen) equals the plain
oracle (oracle.knn) over the materialised corpus: same generator rows, fp16
rounding (numpy's astype, round to nearest even, overflow to inf), planted
rows and (distance, row) order.  The full-size GPU tests (configs[3]/[4]:
246 / 154 GB corpora) check against knn_gen, which never holds the corpus."""

from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as O


@pytest.mark.parametrize("dtype", [np.float32, np.float16])
@pytest.mark.parametrize("metric", ["l2", "cosine", "inner_product"])
def test_knn_gen_equals_knn(dtype, metric):
    n, d = 20_011, 96
    x = O.fill_normal(n, d, 5, row_base=100, dtype=dtype)
    q = O.fill_normal(3, d, 9)
    with np.errstate(over="ignore"):
        planted = {7: q[0] * 3, n - 1: q[1] * 1e6, 4096: np.full(d, 6e-8, np.float32)}
        x2 = x.copy()
        for r, v in planted.items():
            x2[r] = np.asarray(v, dtype=np.float32).astype(dtype)
    a = O.knn(x2, q, metric, 50, row_base=100)
    b = O.knn_gen(n, d, 5, q, metric, 50, row_base=100, dtype=dtype, overrides=planted)
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[0], b[0])


def test_knn_gen_clustered_and_chunk_edges():
    n, d = 3 * 1024 + 5, 40
    x = O.fill_normal(n, d, 2, row_base=1_000_000, cluster=1000)
    q = O.fill_normal(2, d, 3)
    a = O.knn(x, q, "l2", 30, row_base=1_000_000)
    b = O.knn_gen(n, d, 2, q, "l2", 30, row_base=1_000_000, cluster=1000)
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[0], b[0])
