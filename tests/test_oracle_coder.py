"""The coder oracle (oracle/coder.py) against the reference's own outputs
(tests/golden/g5_coder.npz, made by tests/golden/make_golden_coder.py from
src/fenix/io/coder/coder.py).  CPU only."""

from __future__ import annotations

import json

import numpy as np
import pytest

from oracle import coder as OC
from oracle.oracle import fill_normal


@pytest.fixture(scope="module")
def g5(golden_dir):
    g = np.load(f"{golden_dir}/g5_coder.npz")
    return g, json.loads(str(g["meta"]))


def _call_inputs(meta):
    c = meta["call"]
    cw = fill_normal(c["nb"] * c["ks"], c["D"], seed=c["cw_seed"]).reshape(c["nb"], c["ks"], c["D"])
    x = fill_normal(c["n"], c["D"], seed=c["x_seed"], cluster=c["x_cluster"])
    t = fill_normal(c["nt"], c["D"], seed=c["t_seed"])
    return cw, x, t


@pytest.mark.parametrize("metric", ["l2", "cosine", "dot"])
def test_update_matches_reference(g5, metric):
    g, meta = g5
    u = meta["update"]
    q = fill_normal(u["nb"] * u["ks"], u["D"], seed=u["q_seed"]).reshape(u["nb"], u["ks"], u["D"])
    v = fill_normal(u["nb"] * u["bs"], u["D"], seed=u["v_seed"], cluster=u["v_cluster"])
    out = OC.update_all(q, v.reshape(u["nb"], u["bs"], u["D"]), metric)
    ref = g[f"update_{metric}"]
    # float32 reference vs float64 restatement: same assignments, means to f32 rounding
    assert np.abs(out - ref).max() <= 1e-6 * np.abs(ref).max()


@pytest.mark.parametrize("metric", ["l2", "cosine", "dot"])
def test_call_codes_probes_order_match_reference(g5, metric):
    g, meta = g5
    cw, x, t = _call_inputs(meta)
    np.testing.assert_array_equal(OC.call(x, cw, metric, 1)[:, 0], g[f"call_codes_{metric}"])
    p = meta["call"]["probes"]
    np.testing.assert_array_equal(OC.call(t, cw, metric, p), g[f"call_probe_{metric}"])
    np.testing.assert_array_equal(OC.call(t, cw, metric, None), g[f"call_sort_{metric}"])


@pytest.mark.parametrize("metric", ["l2", "cosine", "dot"])
def test_make_matches_reference(g5, metric):
    g, meta = g5
    mk = meta["make"]
    x = fill_normal(mk["n"], mk["D"], seed=mk["x_seed"], cluster=mk["x_cluster"])
    np.random.seed(mk["np_seed"])
    out = OC.make(x, metric, mk["codebook_size"], mk["num_codebooks"], mk["batch_size"],
                  mk["num_epochs"])
    ref = g[f"make_{metric}"]
    assert out.shape == ref.shape
    assert np.abs(out - ref).max() <= 1e-6 * np.abs(ref).max()


def test_composite_digits():
    dg = OC.digits(3, 4)
    c = np.arange(64)
    np.testing.assert_array_equal(dg[0] * 16 + dg[1] * 4 + dg[2], c)
