"""bench.py's result checks, on the CPU: the planted rows it verifies come
back first and in rank order under every metric (checked with the float64
oracle over a small shard set), and its host merge of gathered lists orders
by (distance, row) with NaN last and empty slots dropped -- the order
fx_topk_merge must reproduce bit for bit (tests/test_gpu_distributed.py)."""

from __future__ import annotations

import numpy as np
import pytest
import torch

import bench
from oracle import oracle as O


@pytest.mark.parametrize("metric", ["l2", "cosine", "inner_product"])
@pytest.mark.parametrize("world", [1, 3])
def test_planted_rows_rank_first_in_rank_order(metric, world):
    n, d, k = 4_000, 64, 10
    q = torch.from_numpy(O.fill_normal(1, d, seed=1))
    shards, planted = [], []
    for rank in range(world):
        x = torch.from_numpy(O.fill_normal(n, d, seed=100 + rank))
        planted.append(rank * n + bench.plant_rows(x, q, metric, rank, world))
        shards.append(x.numpy())
    allx = np.concatenate(shards)
    od, orow = O.knn(allx, q.numpy(), metric, k)
    assert orow[0, :world].tolist() == planted


def test_host_merge_orders_by_distance_then_row_nan_last():
    k = 4
    gd = np.array([[[0.5, 0.25, np.nan, 1.0], [0.25, 0.75, 2.0, np.nan]]], np.float32)
    gr = np.array([[[7, 9, 3, 1], [4, -1, 2, 5]]], np.int64)
    od, orow = bench.host_merge(gd, gr, k)
    # 0.25 (rows 4 and 9: row order), 0.5 (7), 1.0 (1); row -1 dropped, NaNs last
    assert orow[0].tolist() == [4, 9, 7, 1]
    np.testing.assert_array_equal(od[0], np.array([0.25, 0.25, 0.5, 1.0], np.float32))
    # all seven live entries: 2.0 (row 2), then the NaNs by row (3, 5)
    od, orow = bench.host_merge(gd, gr, 7)
    assert orow[0].tolist() == [4, 9, 7, 1, 2, 3, 5]
    assert od[0, 4] == 2.0 and np.isnan(od[0, 5]) and np.isnan(od[0, 6])
    # more slots than live entries: the rest stay empty (row -1)
    od, orow = bench.host_merge(gd, gr, 8)
    assert orow[0, 7] == -1
