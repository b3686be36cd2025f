"""Golden vectors for the coded index, generated from the reference (nrlugg/fenix).

Run ONLY in the build container, where the reference checkout exists:

    python tests/golden/make_golden_coder.py

Records what the reference returns from

* ``fenix.io.coder.update`` under ``torch.vmap`` (src/fenix/io/coder/coder.py:53-65,
  the training step ``make`` applies, :95, :118) for every metric;
* ``fenix.io.coder.call`` (coder.py:143-194): composite codes of many rows with
  ``maxval=1`` (how index.make encodes a table, index.py:46-49), the ``probes``
  nearest composites of single targets (index.py:117-121) and the full argsort
  (``maxval=None``);
* ``fenix.io.coder.make`` (coder.py:94-127): the trained codebooks for a fixed
  ``np.random.seed``.  ``make`` wraps ``update`` in ``torch.compile``, which fails
  in this container, so ``torch.compile`` is replaced by the
  identity while it runs; and ``torch.save`` is intercepted to capture the
  coding instead of writing a pickle (its ``column`` entry is a pickled
  ``pa.DataType`` that ``torch.load(weights_only=True)`` refuses).

Inputs come from ``oracle.fill_normal`` (portable generator); only outputs and
the generator parameters are stored (``tests/golden/g5_coder.npz``).
"""

from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np
import pyarrow as pa

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from oracle.oracle import fill_normal  # noqa: E402
from make_golden import _import_fenix  # noqa: E402

METRICS = ["l2", "cosine", "dot"]


def main() -> None:
    import torch

    fenix = _import_fenix()
    import importlib

    C = importlib.import_module("fenix.io.coder.coder")  # the module (update is not re-exported)
    import fenix.io.table as T

    rec = {}
    meta = {"metrics": METRICS}

    # -- update (one vmapped k-means step), D=32, nb=2, ks=8, bs=256, clustered
    D, nb, ks, bs = 32, 2, 8, 256
    q = fill_normal(nb * ks, D, seed=101).reshape(nb, ks, D)
    v = fill_normal(nb * bs, D, seed=102, cluster=32).reshape(nb, bs, D)
    meta["update"] = {"D": D, "nb": nb, "ks": ks, "bs": bs, "q_seed": 101, "v_seed": 102,
                      "v_cluster": 32}
    step = torch.vmap(C.update)
    for m in METRICS:
        out = step(torch.from_numpy(q), torch.from_numpy(v), metric=m)
        rec[f"update_{m}"] = out.numpy()

    # -- call: composite codes, probes, argsort
    D, nb, ks, n = 48, 3, 5, 2000
    cw = fill_normal(nb * ks, D, seed=111).reshape(nb, ks, D)
    x = fill_normal(n, D, seed=112, cluster=100)
    t = fill_normal(4, D, seed=113)
    meta["call"] = {"D": D, "nb": nb, "ks": ks, "n": n, "cw_seed": 111, "x_seed": 112,
                    "x_cluster": 100, "t_seed": 113, "nt": 4, "probes": 16}
    vt = pa.list_(pa.float32(), D)
    for m in METRICS:
        coding = {"tensor": torch.from_numpy(cw), "column": vt,
                  "config": {"metric": m, "codebook_size": ks, "num_codebooks": nb,
                             "batch_size": 1, "num_epochs": 1}}
        rec[f"call_codes_{m}"] = C.call(x, coding, 1)[:, 0].astype(np.int64)
        rec[f"call_probe_{m}"] = np.stack([C.call(t[i : i + 1], coding, 16)[0] for i in range(4)])
        rec[f"call_sort_{m}"] = np.stack([C.call(t[i : i + 1], coding, None)[0] for i in range(4)])

    # -- make: trained codebooks for a fixed seed
    D, n = 64, 20_000
    cfg = {"codebook_size": 8, "num_codebooks": 2, "batch_size": 512, "num_epochs": 3}
    meta["make"] = {"D": D, "n": n, "x_seed": 121, "x_cluster": 1000, "np_seed": 7, **cfg}
    x = fill_normal(n, D, seed=121, cluster=1000)
    ids = pa.array(np.arange(n, dtype=np.int64))
    arr = pa.FixedSizeListArray.from_arrays(pa.array(x.ravel()), list_size=D)
    table = pa.table({"id": ids, "vector": arr}).to_batches(max_chunksize=1000)
    saved = {}
    real_compile, real_save = torch.compile, C.torch.save

    def capture(obj, f):
        saved["tensor"] = obj["tensor"].detach().clone()

    with tempfile.TemporaryDirectory() as root:
        T.make(root, "g/src", pa.RecordBatchReader.from_batches(table[0].schema, table))
        for m in METRICS:
            torch.compile = lambda f, *a, **k: f
            C.torch.save = capture
            try:
                np.random.seed(7)
                try:
                    C.make(root, f"g/{m}", "g/src", "vector", {"metric": m, **cfg})
                except Exception:  # load() of the (never written) file
                    pass
            finally:
                torch.compile, C.torch.save = real_compile, real_save
            rec[f"make_{m}"] = saved.pop("tensor").numpy()

    np.savez_compressed(os.path.join(HERE, "g5_coder.npz"), meta=json.dumps(meta), **rec)
    print("wrote g5_coder.npz:", sorted(rec))


if __name__ == "__main__":
    main()
