"""Metric kernels behind ``distance`` — the arithmetic of the search path.

Mirrors ``distance`` of src/fenix/io/coder/coder.py:38-50:

* ``euclidean`` / ``l2``       sqrt(sum (u-v)^2)          (torch.cdist, :39-40)
* ``cosine``                   0.5 - 0.5 * normalize(u) . normalize(v)   (:42-45)
* ``dot`` / ``inner_product``  -(u . v)                   (:47-48)
* anything else                ``ValueError()``           (:50)

Here every pair is evaluated by the gfx950 scan kernel (``fx_knn_distances``)
with direct differences in f32 — never the ``|u|^2+|v|^2-2uv`` expansion that
cdist uses above 25 rows, which loses all precision at near-duplicates.
Inputs may live on the CPU (they are copied to HBM) or on the GPU; the result
is returned on ``v``'s device with ``v``'s dtype, shape ``[rows(u), rows(v)]``
(the reference squeezes the batch axis at its call site, index.py:142-149).

Product-quantiser training (coder.py:53-127) and coded-index lookup
(coder.py:143-194) are outside the MI355X hot path.
"""

from __future__ import annotations

import torch
from torch import Tensor

from .. import _lib
from ..engine import Engine, Shard

METRICS = frozenset(_lib.METRICS)


def metric_id(metric: str) -> int:
    try:
        return _lib.METRICS[metric]
    except (KeyError, TypeError):
        raise ValueError() from None


def distance(u: Tensor, v: Tensor, metric: str) -> Tensor:
    m = metric_id(metric)
    if v.dim() != 2:
        raise ValueError("v must be [rows, D]")
    if v.dtype not in (torch.float32, torch.float16):
        raise NotImplementedError(f"fenix_amd scans float32/float16 embeddings, got {v.dtype}")
    uu = u.reshape(-1, u.shape[-1])
    if uu.shape[-1] != v.shape[-1]:
        raise ValueError(f"dimension mismatch {uu.shape[-1]} != {v.shape[-1]}")
    eng = Engine.get()
    dv = v.to(eng.device).contiguous()
    # the query takes the column's value type first (index.py:111 casts it)
    q = uu.to(eng.device).to(v.dtype).to(torch.float32).contiguous()
    out = eng.distances(Shard(dv, 0), q, m)
    out = out.to(v.dtype).reshape(*u.shape[:-1], v.shape[0])
    return out.to(v.device)
