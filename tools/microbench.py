"""In-process A/B of scan-kernel variants, merge settings and the measured
stream-read ceiling (interleaved rounds, one process: cdna_hip_programming.md
§5.4 rule 24).  Not part of the product; results go to gpurun_out/.

    python tools/microbench.py [--n 10000000] [--d 768] [--rounds 3] [--iters 10]
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fenix_amd import _lib  # noqa: E402
from fenix_amd.engine import Engine, Shard  # noqa: E402


def bind(path):
    L = ctypes.CDLL(path)
    i64, sz, vp, ci = ctypes.c_int64, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int
    L.fx_knn_workspace_bytes.argtypes = [i64, i64, ci, i64, i64, ctypes.POINTER(sz)]
    L.fx_knn_scan.argtypes = [vp, ci, i64, i64, i64, vp, i64, ci, i64, vp, vp, sz, vp]
    L.fx_knn_reduce.argtypes = [vp, ci, i64, i64, i64, vp, i64, ci, i64, vp, vp, sz, vp, vp, vp]
    L.fx_last_error.restype = ctypes.c_char_p
    return L


def timed(fn, iters):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(iters)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in evs]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--d", type=int, default=768)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--metric", type=int, default=0)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--occ", default="0,2,3,4")
    p.add_argument("--groups", default="0,8,16,32")
    p.add_argument("--variants", action="store_true")
    p.add_argument("--nq", type=int, default=1)
    p.add_argument("--sweep", default="", help="d:dtype list, e.g. 128:f32,1536:f16 (occ only)")
    p.add_argument("--interleave", default="", help="FX_SCAN_INTERLEAVE values to A/B, e.g. 0,1")
    a = p.parse_args()
    if a.sweep:
        return sweep(a)
    eng = Engine.get(torch.device("cuda", 0))
    n, d, k = a.n, a.d, a.k
    x = torch.empty((n, d), dtype=torch.float32, device=eng.device)
    eng.fill(x, seed=0)
    nq = a.nq
    q = torch.empty((nq, d), dtype=torch.float32, device=eng.device)
    eng.fill(q, seed=1)
    nbytes = n * d * 4
    stream = torch.cuda.current_stream().cuda_stream
    libs = {"main(nt1,u1)": _lib.LIB_PATH}
    for f in sorted(os.listdir(os.path.join(ROOT, "tools", "build"))):
        if f.startswith("libfenix_knn_"):
            libs[f[len("libfenix_knn_"):-3]] = os.path.join(ROOT, "tools", "build", f)
    bound = {name: bind(path) for name, path in libs.items()}
    results = {}

    def scan_variant(L, occ, il=None):
        os.environ["FX_SCAN_BLOCKS_PER_CU"] = "8"  # max blocks = largest workspace
        need = ctypes.c_size_t(0)
        assert L.fx_knn_workspace_bytes(n, d, 0, nq, k, ctypes.byref(need)) == 0
        os.environ.pop("FX_SCAN_BLOCKS_PER_CU", None)
        ws = torch.empty(need.value, dtype=torch.uint8, device=eng.device)

        def run():
            if occ:
                os.environ["FX_SCAN_BLOCKS_PER_CU"] = str(occ)
            else:
                os.environ.pop("FX_SCAN_BLOCKS_PER_CU", None)
            os.environ.pop("FX_SCAN_INTERLEAVE", None)
            os.environ.pop("FX_SCAN_PIPE", None)
            if il is not None:  # "1" / "0" interleave, "1p" / "0p": also FX_SCAN_PIPE=0
                os.environ["FX_SCAN_INTERLEAVE"] = il[0]
                if il.endswith("p"):
                    os.environ["FX_SCAN_PIPE"] = "0"
            rc = L.fx_knn_scan(x.data_ptr(), 0, n, d, 0, q.data_ptr(), nq, a.metric, k, None,
                               ws.data_ptr(), ws.numel(), stream)
            assert rc == 0, L.fx_last_error()
        return run

    sr = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libstream_read.so"))
    sr.stream_read_launch.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    sink = torch.zeros(1 << 16, dtype=torch.int32, device=eng.device)

    def stream_variant(blocks, nt):
        def run():
            assert sr.stream_read_launch(x.data_ptr(), nbytes, sink.data_ptr(), blocks, nt,
                                         stream) == 0
        return run

    variants = {}
    ils = a.interleave.split(",") if a.interleave else [None]
    for name, L in bound.items():
        for occ in [int(v) for v in a.occ.split(",")]:
            for il in ils:
                tag = "" if il is None else f",il={il}"
                variants[f"scan[{name},occ={occ or 'max'}{tag}]"] = scan_variant(L, occ, il)
    for blocks in (1024, 2048, 4096, 8192) if nq == 1 else ():
        for nt in (0, 1):
            variants[f"stream_read[blocks={blocks},nt={nt}]"] = stream_variant(blocks, nt)
    for r in range(a.rounds):
        for name, fn in variants.items():
            if name.startswith("scan"):
                fn = variants[name]
            ts = timed(fn, a.iters)
            results.setdefault(name, []).extend(ts)
        print(f"round {r} done", flush=True)
    os.environ.pop("FX_SCAN_BLOCKS_PER_CU", None)
    os.environ.pop("FX_SCAN_INTERLEAVE", None)
    os.environ.pop("FX_SCAN_PIPE", None)

    # merge (reduce) settings on the default scan
    if nq > 1:
        a.groups = "0"
    shard = Shard(x, 0)
    od = torch.empty((1, k), dtype=torch.float32, device=eng.device)
    orow = torch.empty((1, k), dtype=torch.int64, device=eng.device)
    for g in [int(v) for v in a.groups.split(",")]:
        if g:
            os.environ["FX_MERGE_GROUP"] = str(g)
        else:
            os.environ.pop("FX_MERGE_GROUP", None)
        ws = eng.scan(shard, q, a.metric, k)
        ts = timed(lambda: eng.reduce(shard, q, a.metric, k, ws, od, orow), a.iters * 2)
        results[f"reduce[group={g or 'auto'}]"] = ts
    os.environ.pop("FX_MERGE_GROUP", None)

    summary = {}
    for name, ts in results.items():
        med = float(np.median(ts))
        entry = {"median_ms": med, "min_ms": float(np.min(ts))}
        if name.startswith(("scan", "stream")):
            if nq > 1:
                entry["TFLOPs_median"] = 2.0 * n * nq * d / (med * 1e-3) / 1e12
            entry["GBps_median"] = nbytes / (med * 1e-3) / 1e9
            entry["GBps_best"] = nbytes / (np.min(ts) * 1e-3) / 1e9
        summary[name] = entry
        print(f"{name:48s} {json.dumps(entry)}", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "microbench.json"), "w") as f:
        json.dump(summary, f, indent=1)


def sweep(a):
    """Occupancy sweep of the main library's scan over several shapes (~30 GB each)."""
    eng = Engine.get(torch.device("cuda", 0))
    libs = {"main": bind(_lib.LIB_PATH)}
    if a.variants:
        for f in sorted(os.listdir(os.path.join(ROOT, "tools", "build"))):
            if f.startswith("libfenix_knn_"):
                libs[f[len("libfenix_knn_"):-3]] = bind(os.path.join(ROOT, "tools", "build", f))
    L = libs["main"]
    stream = torch.cuda.current_stream().cuda_stream
    summary = {}
    for spec in a.sweep.split(","):
        ds, dt = spec.split(":")
        d = int(ds)
        tdt, es, code = (torch.float32, 4, 0) if dt == "f32" else (torch.float16, 2, 1)
        n = int(30.72e9 // (d * es))
        x = torch.empty((n, d), dtype=tdt, device=eng.device)
        eng.fill(x, seed=0)
        q = torch.empty((1, d), dtype=torch.float32, device=eng.device)
        eng.fill(q, seed=1)
        os.environ.pop("FX_SCAN_BLOCKS_PER_CU", None)
        need = 0
        for Lv in libs.values():
            nb = ctypes.c_size_t(0)
            assert Lv.fx_knn_workspace_bytes(n, d, code, 1, a.k, ctypes.byref(nb)) == 0
            need = max(need, nb.value)
        ws = torch.empty(need, dtype=torch.uint8, device=eng.device)
        res = {}
        for r in range(a.rounds):
            for (lname, L), occ in [(lv, o) for lv in libs.items()
                                    for o in [int(v) for v in a.occ.split(",")]]:
                def run(occ=occ, L=L):
                    if occ:
                        os.environ["FX_SCAN_BLOCKS_PER_CU"] = str(occ)
                    else:
                        os.environ.pop("FX_SCAN_BLOCKS_PER_CU", None)
                    rc = L.fx_knn_scan(x.data_ptr(), code, n, d, 0, q.data_ptr(), 1, a.metric,
                                       a.k, None, ws.data_ptr(), ws.numel(), stream)
                    assert rc == 0, L.fx_last_error()
                res.setdefault((lname, occ), []).extend(timed(run, a.iters))
        for (lname, occ), ts in res.items():
            med = float(np.median(ts))
            key = f"scan[{lname},d={d},{dt},n={n},occ={occ or 'max'}]"
            summary[key] = {"median_ms": med, "GBps_median": n * d * es / (med * 1e-3) / 1e9}
            print(f"{key:48s} {json.dumps(summary[key])}", flush=True)
        del x, ws
        torch.cuda.empty_cache()
    os.environ.pop("FX_SCAN_BLOCKS_PER_CU", None)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "microbench_sweep.json"), "w") as f:
        json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
