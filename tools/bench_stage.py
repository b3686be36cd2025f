"""Host -> HBM staging throughput of an Arrow column (engine.stage_column):
the one-time cost per file version before the first search.

    python tools/bench_stage.py --n 4000000 --d 768
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402
import torch  # noqa: E402

from fenix_amd import engine  # noqa: E402


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=4_000_000)
    p.add_argument("--d", type=int, default=768)
    p.add_argument("--chunk", type=int, default=1000)
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    eng = engine.Engine.get(torch.device("cuda", 0))
    x = np.empty((a.n, a.d), dtype=np.float32)
    tmp = torch.empty((1_000_000, a.d), dtype=torch.float32, device=eng.device)
    for s in range(0, a.n, tmp.shape[0]):
        m = min(tmp.shape[0], a.n - s)
        eng.fill(tmp[:m], seed=0, row_base=s)
        x[s : s + m] = tmp[:m].cpu().numpy()
    del tmp
    flat = pa.array(x.reshape(-1))
    chunks = [pa.FixedSizeListArray.from_arrays(flat.slice(s * a.d, min(a.chunk, a.n - s) * a.d),
                                                a.d) for s in range(0, a.n, a.chunk)]
    col = pa.chunked_array(chunks)
    ts = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = engine.stage_column(col, eng.device)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
        ok = bool(torch.equal(out[-1].cpu(), torch.from_numpy(x[-1])))
        del out
    gb = x.nbytes / 1e9
    print(json.dumps({"rows": a.n, "d": a.d, "chunk_rows": a.chunk, "gbytes": gb,
                      "seconds": ts, "gb_per_s": gb / min(ts), "last_row_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
