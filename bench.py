"""Benchmark of the fenix brute-force kNN hot path on MI355X.

Workload (BASELINE.json configs[1], the headline metric's config): one query,
10M x 768 float32 rows per GPU, L2, k=100, corpus resident in HBM.  One
"step" = one exact search over every row of this rank's shard, merge to the
final sorted k, and for N > 1 the RCCL all-gather of the per-rank top-k plus
the final merge (weak scaling: 10M rows per GPU, so N=8 is configs[3], 80M
rows).

The headline (``value``, ``ms_per_step``, ``roofline``) is the exact fused
f32 scan that reads every row, SURVEY §8(d): 3 072 B per vector, 30.72 GB per
search.  The product default for the same single query streams a resident
int8 filter image instead and rescores its candidates exactly (bit-identical
results); it is timed as a second leg and reported under
``accelerated_exact`` with the image's own bytes.  Batches (``--nq`` > 1,
configs[2]) run the product path in the headline, priced over the image bytes
(``roofline.bytes_basis``).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rows ROWS] [--d D]
                    [--k K] [--nq Q] [--metric l2|cosine|inner_product]
                    [--dtype f32|f16|qu8] [--cluster C] [--query normal|near]
                    [--no-accelerated] [--no-cpu-baseline] [--strong-rows R]
                    [--serve-devices 0,1,...]

For N > 1 the line also carries ``strong`` (BASELINE's fixed 10M-row corpus
split over the N ranks) and ``serve`` (rank 0 alone: one process searching a
row shard on every device through engine._search_all, the path a Flight
server runs, with the RCCL all-gather and with peer copies).

Every leg checks its result: sorted and complete, one planted row per rank
returned first in rank order (global row numbering), for N > 1 the merge
equal to the host's merge of the gathered lists, and the accelerated leg
equal to the exact scan bit for bit.

``--gpus N`` under a launcher (torch.distributed.run sets WORLD_SIZE) must
equal the world size; without one, N > 1 starts the N ranks itself (a
torch.distributed.run child, before this process touches a GPU).

Prints ONE JSON line on rank 0 (see DESIGN.md §6 for every field).
"""

from __future__ import annotations

import argparse
import datetime
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md chip table
MFMA_F16_PEAK_TFS = 2500.0  # dense fp16/bf16 matrix peak, same table

METRIC = "vectors/sec + %HBM roofline, 10M×768 f32 L2 kNN k=100 at 1/2/4/8 GPU"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--rows", dest="n", type=int, default=10_000_000, help="rows per GPU")
    p.add_argument("--d", type=int, default=768)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--nq", type=int, default=1)
    p.add_argument("--metric", default="l2")
    p.add_argument("--dtype", default="f32", choices=["f32", "f16", "qu8"],
                   help="qu8: quint8 codes (ex/arrow/quint8), scanned by fx_knn_search_ex")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-verify", action="store_true",
                   help="skip the result checks and the planted rows (diagnostic builds)")
    p.add_argument("--no-batch-leg", action="store_true",
                   help="skip the configs[2] batch leg (256 cosine queries over the same image)")
    p.add_argument("--no-accelerated", action="store_true",
                   help="skip the filter-image leg (profiling the exact scan alone)")
    p.add_argument("--cluster", type=int, default=0,
                   help="rows clustered per C rows, x + 10 x0 (tests/test_flight.py:21-22)")
    p.add_argument("--query", default="normal", choices=["normal", "near"],
                   help="near: the query is corpus row n/3 + N(0,1)/2")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    p.add_argument("--cpu-rows", type=int, default=1_000_000)
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                   help="library option (fx_set_option), e.g. batch_sample_ratio=20; sweeps only")
    p.add_argument("--strong-rows", type=int, default=-1,
                   help="N > 1: also time the exact search of this many rows in total, split "
                        "over the N ranks (strong scaling; default --rows, i.e. configs[1]'s "
                        "10M); 0 skips it")
    p.add_argument("--serve-devices", default="",
                   help="comma-separated ordinals: also time one process searching row shards "
                        "on these devices (engine._search_all, the Flight server's path); "
                        "default at N > 1: every rank's device, from rank 0")
    return p.parse_args()


def check_frac(name: str, frac: float) -> float:
    """A roofline fraction above 1 means the timed span did not bracket the
    work it is priced on: fail loudly instead of printing it."""
    if not frac <= 1.0:
        sys.exit(f"bench.py: {name} = {frac:.3f} > 1: the timed span misses part of the work")
    return frac


def cpu_baseline(args):
    """Oracle C restatement (float32 direct formulas, OpenMP, heap top-k) on a
    bounded sample of the same workload, timed on this host's cores."""
    from oracle import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = min(threads, len(os.sched_getaffinity(0)))
    rows = min(args.cpu_rows, args.n)
    x = np.empty((rows, args.d), dtype=np.float32)
    O.lib().fx_ref_fill(O._ptr(x), rows, args.d, 0, 0, 0)
    if args.dtype == "f16":
        x = x.astype(np.float16)
    if args.dtype == "qu8":  # the CPU port scans the dequantised float32 values
        x = O.dequantize(np.clip(np.rint(x / QU8_SCALE) + QU8_ZP, 0, 127), QU8_SCALE, QU8_ZP)
    q = O.fill_normal(1, args.d, 1)
    O.knn(x[: min(rows, 10000)], q, args.metric, args.k, precision=32, threads=threads)
    done, t0 = 0, time.perf_counter()
    while True:
        O.knn(x, q, args.metric, args.k, precision=32, threads=threads)
        done += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds:
            break
    return {
        "value": rows * done / el,
        "unit": "vectors/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{rows}x{args.d} {args.dtype} {args.metric} k={args.k}, {done} single-query "
        f"searches in {el:.1f}s (oracle/knn_ref.c precision=32, same generator)",
        "reference_algorithm": torch_cpu_baseline(args, x, q, threads),
    }


def torch_cpu_baseline(args, x, q, threads):
    """The reference's own arithmetic on the CPU: coder.distance (torch.cdist /
    -u@v.T / normalised matmul, src/fenix/io/coder/coder.py:38-50) over the
    sample + torch.topk in place of select_k_unstable (index.py:166), without
    the per-chunk Arrow UDF and Table.take overheads the reference adds."""
    xt = torch.from_numpy(np.asarray(x, dtype=np.float32))
    qt = torch.from_numpy(np.asarray(q, dtype=np.float32))
    torch.set_num_threads(threads)

    def one():
        if args.metric in ("l2", "euclidean"):
            d = torch.cdist(qt, xt)
        elif args.metric == "cosine":
            d = 0.5 - 0.5 * torch.nn.functional.normalize(qt, dim=-1) @ \
                torch.nn.functional.normalize(xt, dim=-1).T
        else:
            d = -qt @ xt.T
        return torch.topk(d, args.k, largest=False)

    one()
    done, t0 = 0, time.perf_counter()
    while True:
        one()
        done += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds / 2:
            break
    return {"value": x.shape[0] * done / el, "unit": "vectors/s", "cores": threads,
            "sample": f"same sample, torch {torch.__version__} CPU, {done} searches in {el:.1f}s"}


# quint8 bench corpus: the generator's N(0,1) rows coded with a fixed per-tensor
# affine map over its range (|x| <= 2*sqrt(3)), codes 0..127 (reduce_range)
QU8_SCALE = float(np.float32(4 * 3**0.5 / 127))
QU8_ZP = 64


def pmc_traffic(workload_tag, kernel, lib_sha):
    """HBM bytes per scan launch from a committed rocprofv3 --pmc summary
    (profiles/*pmc*.json, FETCH_SIZE x2 gfx950 correction already applied,
    tools/summarize_profiles.py) of THIS build: the summary must carry the
    SHA-256 of the library it measured, equal to the loaded one's, else the
    traffic is unknown (None) — a kernel change makes an old pass stale."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            with open(path) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        if (rec.get("workload") == workload_tag and "hbm_bytes_per_launch" in rec
                and kernel in rec.get("kernel", "") and rec.get("library_sha") == lib_sha):
            return float(rec["hbm_bytes_per_launch"])
    return None


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """``--gpus N`` without a launcher: start N ranks (one per GPU) as a
    torch.distributed.run child on 127.0.0.1 and return its exit code.  Runs
    before this process touches the GPU, and starts a child instead of
    re-executing itself."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.run(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1")).returncode


def plant_rows(x: torch.Tensor, q: torch.Tensor, metric: str, rank: int, world: int):
    """Plant one row per rank that must rank ``rank``-th of the merged top-k:
    L2 / cosine: q + (rank+1)/16 e_0 (distance (rank+1)/16 for L2, growing
    with the offset for cosine); inner product: (1000 - rank) q.  Returns the
    local row.  (One row of the shard: the workload is unchanged otherwise.)"""
    p = (rank * 7919 + 12345) % x.shape[0]
    v = q[0].to(torch.float32).clone()
    if metric in ("inner_product", "dot"):
        v = v * float(1000 - rank)
    else:
        v[0] += (rank + 1) / 16.0
    x[p] = v.to(x.dtype)
    return p


def host_merge(gd: np.ndarray, gr: np.ndarray, k: int):
    """(distance, row) merge of gathered [nq, parts, kin] lists on the host:
    the order fx_topk_merge must reproduce bit for bit."""
    nq = gd.shape[0]
    od = np.empty((nq, k), np.float32)
    orow = np.empty((nq, k), np.int64)
    for i in range(nq):
        dd = gd[i].ravel().astype(np.float64)
        rr = gr[i].ravel()
        keep = rr >= 0
        dd, rr = dd[keep], rr[keep]
        o = np.lexsort((rr, np.where(np.isnan(dd), np.inf, dd)))[:k]
        od[i, : len(o)], orow[i, : len(o)] = dd[o], rr[o]
        orow[i, len(o):] = -1
    return od, orow


def main():
    args = parse()
    if args.strong_rows < 0:
        args.strong_rows = args.n
    if args.gpus < 1:
        sys.exit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; --dist-backend gloo lets several ranks share one GPU
    # (multi-rank rehearsal on a single-GPU box: RCCL refuses duplicate GPUs)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    gloo = args.dist_backend == "gloo"
    # FENIX_AMD_BENCH_DIST=1 runs the N > 1 code path (process group, all-gather,
    # barriers, max-over-ranks) at any world size: the one-GPU box exercises
    # the RCCL calls the 8-GPU run makes
    use_dist = world > 1 or os.environ.get("FENIX_AMD_BENCH_DIST") == "1"
    if use_dist:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)

    from fenix_amd import _lib
    from fenix_amd.distributed import allgather_topk, shard_rows
    from fenix_amd.engine import Engine, Shard

    eng = Engine.get(device)
    for o in args.opt:
        name, value = o.split("=", 1)
        _lib.set_option(name, int(value))
    qu8 = args.dtype == "qu8"
    tdt = {"f32": torch.float32, "f16": torch.float16, "qu8": torch.uint8}[args.dtype]
    esize = {"f32": 4, "f16": 2, "qu8": 1}[args.dtype]
    metric = _lib.METRICS[args.metric]
    n, d, k, nq = args.n, args.d, args.k, args.nq
    row_base = rank * n
    x = torch.empty((n, d), dtype=tdt, device=device)
    if qu8:  # synthetic codes: generator rows, quantised in 1M-row slices (data prep)
        tmp = torch.empty((1_000_000, d), dtype=torch.float32, device=device)
        for s in range(0, n, tmp.shape[0]):
            m = min(tmp.shape[0], n - s)
            eng.fill(tmp[:m], seed=0, row_base=row_base + s, cluster=args.cluster)
            x[s : s + m] = torch.clamp(torch.round(tmp[:m] / QU8_SCALE) + QU8_ZP, 0, 127).to(tdt)
        del tmp
    else:
        eng.fill(x, seed=0, row_base=row_base, cluster=args.cluster)
    qh = torch.empty((nq, d), dtype=torch.float32 if qu8 else tdt, device=device)
    eng.fill(qh, seed=1)
    if args.query == "near":  # a query inside the corpus's distribution: row n/3 + N(0,1)/2
        qh = (x[n // 3 : n // 3 + 1].to(torch.float32) + 0.5 * qh.to(torch.float32)).to(qh.dtype)
    q = qh.to(torch.float32)
    planted = None
    if not qu8 and not args.no_verify:
        planted = plant_rows(x, q, args.metric, rank, world)
        torch.autograd.graph.increment_version(x)

    def planted_global(g, per_rank=None):
        """Global row of rank g's planted row: rank g holds rows [g n, g n + n)
        (weak scaling), or shard_rows(strong_rows, world, g) (strong)."""
        p = (g * 7919 + 12345) % n
        if per_rank is None:
            return g * n + p
        return shard_rows(per_rank, world, g)[0] + p
    shard = Shard(x, row_base, QU8_SCALE, QU8_ZP) if qu8 else Shard(x, row_base)
    od = torch.empty((nq, k), dtype=torch.float32, device=device)
    orow = torch.empty((nq, k), dtype=torch.int64, device=device)

    def make_step(sh, span):
        """One search of shard ``sh`` (+ the all-gather and final merge for
        N > 1).  ``ev``: HIP events on the stream the launches are queued on,
        bracketing the scan launch alone (``span="scan"``, the kernel the
        headline's roofline prices) or every launch of the search, scan and
        reduce (``span="search"``: the filter phases, thresholds, rescoring
        and final select of the int8-image path)."""

        def step(ev=None):
            if ev is not None:
                ev[0].record()
            if qu8:  # fx_knn_search_ex: scan + merge in one call (the merge is ~1 % of it)
                with eng.lock:
                    eng.search_shard(sh, q, metric, k, None, od, orow)
            else:
                st = eng.scan(sh, q, metric, k)
            if ev is not None and span == "scan":
                ev[1].record()
            if not qu8:
                eng.reduce(sh, q, metric, k, st, od, orow)
            if ev is not None and span == "search":
                ev[1].record()
            if use_dist:
                if gloo:
                    gd, gr = allgather_topk(od.cpu(), orow.cpu())
                    gd, gr = gd.to(device), gr.to(device)
                else:
                    gd, gr = allgather_topk(od, orow)  # one RCCL all-gather over xGMI
                md, mr = eng.merge(gd, gr, k)
                return md, mr, gd, gr
            return od.clone(), orow.clone(), None, None

        return step

    def timed_leg(step):
        """W untimed warmup steps, then exactly K steps bracketed by a barrier
        and a device synchronisation on both sides; (elapsed s max over ranks,
        mean event-timed span ms max over ranks, last result)."""
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            res = step(ev[i])
        torch.cuda.synchronize()
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        span = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        if use_dist:
            t = torch.tensor([elapsed, span], dtype=torch.float64, device="cpu" if gloo else device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed, span = float(t[0]), float(t[1])
        return elapsed, span, res

    def verify(res, what, per_rank=None):
        """Sorted and complete; the planted rows first, in rank order; for
        N > 1 the merge equals the host's (distance, row) merge of the
        gathered lists, bit for bit.  ``per_rank``: rows per rank when it is
        not ``n`` (the strong-scaling leg's split of a fixed corpus)."""
        if args.no_verify:
            return
        rd, rr = res[0].cpu().numpy(), res[1].cpu().numpy()
        assert (rr >= 0).all() and np.all(np.diff(rd, axis=1) >= 0), f"{what}: result not sorted"
        if planted is not None and k >= world:
            want = np.array([planted_global(g, per_rank) for g in range(world)])
            assert (rr[0, :world] == want).all(), f"{what}: planted rows {rr[0, :world]} != {want}"
        if res[2] is not None:
            hd, hr = host_merge(res[2].cpu().numpy(), res[3].cpu().numpy(), k)
            assert np.array_equal(hr, rr) and np.array_equal(hd.view(np.uint32),
                                                             rd.view(np.uint32)), \
                f"{what}: device merge differs from the host merge of the gathered lists"

    # the filter image (int8 by default) of the product path, built once per
    # corpus version before any timing: batches stream it in the headline
    # leg, a single query in the accelerated leg
    single = nq == 1 and not qu8
    image = None
    image_build_ms = None
    img_bytes = None
    want_image = not qu8 and not (single and args.no_accelerated) and \
        _lib.filter_image_used(n, d, shard.dtype_id, nq, k, metric)
    if want_image:
        b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b0.record()
        built = eng.filter_image(shard, nq, k, metric)[0] is not None
        b1.record()
        torch.cuda.synchronize()
        if built:
            image_build_ms = b0.elapsed_time(b1)
            image = eng._images.get(id(x))
            img_bytes = int(image[1].numel()) * image[1].element_size() + \
                int(image[2].numel()) * 4
    bits = image[0][3] if image is not None else 16

    # The headline: a single query runs the exact fused scan
    # over every row (option single_query_image=0); batches run the product
    # path (the bound filter over the filter image).
    filt = not single and not qu8 and image is not None
    with _lib.options(single_query_image=0) if single else _nullctx():
        elapsed, scan_ms, res = timed_leg(make_step(shard, "search" if filt else "scan"))
    verify(res, "headline")
    head = res

    # strong scaling (BASELINE's metric as worded: one 10M-row corpus at
    # 1/2/4/8 GPUs): the same exact search over strong_rows rows in total,
    # shard_rows(strong_rows, N, rank) per rank (a prefix of this rank's rows)
    strong = None
    if world > 1 and single and args.strong_rows > 0:
        s_base, s_cnt = shard_rows(args.strong_rows, world, rank)
        if s_cnt > n:
            sys.exit(f"--strong-rows {args.strong_rows} needs {s_cnt} rows per rank (> --rows)")
        s_shard = Shard(x[:s_cnt], s_base)
        with _lib.options(single_query_image=0):
            s_el, s_ms, s_res = timed_leg(make_step(s_shard, "scan"))
        # planted rows beyond a rank's prefix are not in the strong corpus
        if all((g * 7919 + 12345) % n < shard_rows(args.strong_rows, world, g)[1]
               for g in range(world)):
            verify(s_res, "strong", per_rank=args.strong_rows)
        s_bytes = s_cnt * d * esize + nq * d * 4
        strong = {
            "scaling": "strong",
            "total_rows": args.strong_rows,
            "rows_per_gpu": s_cnt,
            "ms_per_step": s_el * 1e3 / args.steps,
            "value": args.strong_rows * nq * args.steps / s_el,
            "unit": "vectors/s",
            "kernel_ms": s_ms,
            "frac": check_frac("strong.frac", s_bytes / (s_ms * 1e-3) / 1e9 / HBM_PEAK_GBS),
            "what": "exact fused scan of each rank's 1/N of the corpus + RCCL all-gather + "
                    "merge; ms_per_step includes the gather and merge, kernel_ms the scan only",
        }

    # the product default for the same single query: the int8 filter image +
    # exact rescoring (bit-identical), timed as its own leg
    accel = None
    if single and image is not None:
        a_el, a_ms, res = timed_leg(make_step(shard, "search"))
        verify(res, "accelerated")
        same = bool(np.array_equal(head[1].cpu().numpy(), res[1].cpu().numpy()) and np.array_equal(
            head[0].cpu().numpy().view(np.uint32), res[0].cpu().numpy().view(np.uint32)))
        if not args.no_verify:
            assert same, "the filter-image search differs from the exact scan"
        pass_bytes = img_bytes + nq * d * 4
        a_traffic = pmc_traffic(f"{n}x{d}_{args.dtype}_{args.metric}_k{k}_q{nq}", "filter_img",
                                _lib.library_sha())
        accel = {
            "what": "the product default for this search: int8 filter image + exact rescoring "
                    "of the candidates from the f32 rows (capi.hip filter_phases)",
            "ms_per_step": a_el * 1e3 / args.steps,
            "vectors_per_s": n * world * nq * args.steps / a_el,
            "kernel_ms": a_ms,
            "kernel": "every launch of the search: query prep, fx::q64i::filter_img6_kernel "
                      "(all phases), thresholds, rescoring, final select",
            "image_bytes": img_bytes,
            "image_build_ms": image_build_ms,
            "bytes_per_search": pass_bytes,
            "achieved_gbs_over_image": pass_bytes / (a_ms * 1e-3) / 1e9,
            "frac_over_image": check_frac("accelerated_exact.frac_over_image",
                                          pass_bytes / (a_ms * 1e-3) / 1e9 / HBM_PEAK_GBS),
            "traffic": a_traffic,
            "traffic_over_image": (a_traffic / pass_bytes) if a_traffic else None,
            "bit_identical": same,
            "speedup_vs_headline": elapsed / a_el,
        }

    # configs[2] beside it (BASELINE configs[2]: the same rows, a 256-query
    # cosine batch through the same resident image), one rank only
    batch = None
    if single and image is not None and world == 1 and not args.no_batch_leg:
        batch = batch_leg(eng, shard, image, img_bytes, n, d, k, args)

    total_rows = n * world
    value = total_rows * nq * args.steps / elapsed
    scan_bytes = n * d * esize + nq * d * 4
    algo_bytes = scan_bytes
    tag = f"{n}x{d}_{args.dtype}_{args.metric}_k{k}_q{nq}"
    if filt:
        # a batch streams the filter image and its row terms instead of the
        # rows (the rescoring reads a few thousand rows per query on top)
        scan_bytes = img_bytes + nq * d * 4
    if filt:
        if bits == 8 and nq <= 128:
            kname = "fx::filter_img6_kernel (int8-MFMA bound filter, all sample phases)"
        elif bits == 8 and d <= 768:
            kname = "fx::filter_img8_kernel (int8-MFMA bound filter, queries in registers, all phases)"
        else:
            kname = f"fx::filter_img3_kernel ({'int8' if bits == 8 else 'fp16'}-MFMA bound filter, all sample phases)"
        kname += " + exact rescoring of the candidates"
    elif qu8:
        kname = "fx::scan_kernel<uint8> (quint8 codes dequantised in registers) + merge"
    else:
        kname = "fx::scan_kernel (fused distance + per-wave top-k)"
    traffic = pmc_traffic(tag, "filter_img" if filt else "scan_kernel", _lib.library_sha())
    achieved = scan_bytes / (scan_ms * 1e-3) / 1e9
    roof = {
        "bound": "hbm",
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "traffic": traffic,
        "kernel": kname,
        "kernel_ms": scan_ms,
        "bytes_per_launch": scan_bytes,
        "library_sha": _lib.library_sha(),
        "build": _lib.build_info(),
    }
    if filt:  # the GEMM the filter evaluates, against the dense MFMA peak of its type
        roof["bytes_basis"] = "filter image + row terms (the pass reads these, not the rows)"
        roof["algorithmic_bytes"] = algo_bytes
        # int8 MFMA work is integer ops (TOPS), fp16 work flops (TFLOPS)
        u = "tops" if bits == 8 else "tflops"
        roof[f"mfma_{u}"] = 2.0 * n * nq * d / (scan_ms * 1e-3) / 1e12
        roof[f"mfma_peak_{u}"] = MFMA_F16_PEAK_TFS * (2 if bits == 8 else 1)
    roof["frac"] = check_frac("roofline.frac", roof["achieved"] / roof["peak"])
    for u in ("tops", "tflops"):
        if f"mfma_{u}" in roof:
            check_frac("roofline.mfma", roof[f"mfma_{u}"] / roof[f"mfma_peak_{u}"])

    # the single-process path a Flight server runs over every GPU of the node
    # (engine._search_all): rank 0 alone, while the other ranks wait on the
    # rendezvous store (no GPU kernel of theirs is spinning meanwhile)
    serve = None
    serve_devs = None
    if args.serve_devices and not qu8:
        serve_devs = [int(v) for v in args.serve_devices.split(",")]
    elif world > 1 and single and not qu8 and torch.cuda.device_count() >= world:
        serve_devs = list(range(world))
    if serve_devs is not None and world > 1:
        store = dist.distributed_c10d._get_default_store()
        if rank == 0:
            try:
                serve = serve_leg(eng, serve_devs, n, d, k, metric, q, args,
                                  head if world == len(serve_devs) else None)
            except Exception as e:  # reported in the line; the rank-path legs stand
                serve = {"error": f"{type(e).__name__}: {e}"}
            finally:
                store.set("fx_bench_serve_done", "1")
        else:
            store.wait(["fx_bench_serve_done"], datetime.timedelta(minutes=20))
    elif serve_devs is not None:
        serve = serve_leg(eng, serve_devs, n, d, k, metric, q, args, None)

    # the CPU baseline is timed after every timed region, on rank 0 only; for
    # N > 1 the other ranks wait on the rendezvous store (not a GPU barrier,
    # so no collective kernel of theirs spins meanwhile)
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args)
        finally:
            if world > 1:
                dist.distributed_c10d._get_default_store().set("fx_bench_cpu_done", "1")
    elif world > 1 and not args.no_cpu_baseline:
        dist.distributed_c10d._get_default_store().wait(["fx_bench_cpu_done"],
                                                         datetime.timedelta(minutes=20))

    out = None
    if rank == 0:
        wl = (f"{n // 1_000_000 if n % 1_000_000 == 0 else n}"
              f"{'M' if n % 1_000_000 == 0 else ''}x{d} {args.dtype} {args.metric.upper()} "
              f"kNN k={k}, {'single query' if nq == 1 else f'{nq}-query batch'}, per GPU"
              + (f", clustered x{args.cluster}" if args.cluster else ""))
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "vectors/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic: portable Irwin-Hall(4) N(0,1) generator on device "
                    "(corpus seed 0, query seed 1), corpus resident in HBM"
                    + (f"; rows clustered per {args.cluster} (x + 10 x0, test_flight.py:21-22)"
                       if args.cluster else "")
                    + ("; query = row n/3 + N(0,1)/2" if args.query == "near" else "")
                    + ("" if planted is None else "; one planted row per rank (verified first)"),
            "config": {
                "workload": wl,
                "path": ("exact fused f32 scan over every row (SURVEY 8(d))" if single
                         else "bound filter over the filter image + exact rescoring"
                         if filt else "exact fused scan"),
                "rows_per_gpu": n,
                "total_rows": total_rows,
                "d": d,
                "k": k,
                "queries": nq,
                "metric": args.metric,
                **({"cluster": args.cluster} if args.cluster else {}),
                **({"query": args.query} if args.query != "normal" else {}),
                **({"options": args.opt} if args.opt else {}),
                "parallelism": f"row-shard x{world}, one process per GPU"
                + ((" + gloo all-gather" if gloo else " + RCCL all-gather") if use_dist else "")
                + (f"; strong leg: {args.strong_rows} rows over {world}" if strong else "")
                + (f"; serve leg: one process over devices {serve_devs}, gathers "
                   f"{'/'.join(serve.get('gathers', {}))}" if serve and "gathers" in serve
                   else ""),
            },
            **({"filter_image": {"bits": bits, "bytes": img_bytes, "build_ms": image_build_ms,
                                 "note": "resident beside the corpus, built once per corpus "
                                         "version (not in ms_per_step)"}}
               if image is not None else {}),
            "roofline": roof,
            **({"strong": strong} if strong is not None else {}),
            **({"serve": serve} if serve is not None else {}),
            **({"accelerated_exact": accel} if accel is not None else {}),
            **({"configs2": batch} if batch is not None else {}),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()
    return out


def serve_leg(eng, devs, n, d, k, metric, q, args, rank_result):
    """The Flight server's multi-GPU path (SURVEY §8(e), configs[3]/[4]'s
    deployment): ONE process holding a row shard of n rows on each listed
    device (the same rows and planted rows the one-process-per-GPU ranks
    hold), searched by engine._search_all — every device's exact scan queued
    back to back, then the per-device top-k exchanged over RCCL (one grouped
    all-gather, the default for distinct devices) or peer copies, and merged on
    the first device.  W + K searches per gather mode, timed from the host with
    every device synchronised on both sides.  ``rank_result``: the
    one-process-per-GPU legs' merged result, which each mode must equal bit
    for bit."""
    from fenix_amd import _lib, engine
    from fenix_amd.engine import Engine, Shard

    world = len(devs)
    shards = []
    for g, ordinal in enumerate(devs):
        dv = torch.device("cuda", ordinal)
        with torch.cuda.device(dv):
            e = Engine.get(dv)
            xs = torch.empty((n, d), dtype=torch.float32 if args.dtype == "f32" else torch.float16,
                             device=dv)
            e.fill(xs, seed=0, row_base=g * n, cluster=args.cluster)
            if not args.no_verify:
                plant_rows(xs, q.to(dv), args.metric, g, world)
                torch.autograd.graph.increment_version(xs)
            shards.append(Shard(xs, g * n))

    def sync_all():
        for o in sorted(set(devs)):
            torch.cuda.synchronize(o)

    # distinct devices: both exchanges; an ordinal repeated on one GPU (a
    # rehearsal) merges its shards on that device with no exchange ("none")
    ndev = len(set(devs))
    modes = ["rccl", "p2p"] if ndev == len(devs) and ndev > 1 else ["p2p"] if ndev > 1 else ["none"]
    out = {"devices": devs, "rows_per_device": n, "total_rows": n * world,
           "what": "one process, exact scan per device shard, gather to the first device, "
                   "fx_topk_merge (engine._search_all, the path Flight.search serves)",
           "gathers": {}}
    old = os.environ.get("FENIX_AMD_GATHER")
    try:
        for mode in modes:
            os.environ["FENIX_AMD_GATHER"] = "p2p" if mode == "none" else mode
            before = dict(engine.GATHERS)
            with _lib.options(single_query_image=0):
                for _ in range(args.warmup):
                    engine._search_all(shards, q, metric, k)
                sync_all()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    rd, rr = engine._search_all(shards, q, metric, k)
                sync_all()
                el = time.perf_counter() - t0
            used = {m: engine.GATHERS[m] - before[m] for m in before}
            rec = {"ms_per_step": el * 1e3 / args.steps,
                   "value": n * world * args.steps / el, "unit": "vectors/s",
                   "gathers_used": used}
            if mode != "none" and used.get(mode, 0) != args.warmup + args.steps:
                raise RuntimeError(f"serve leg: asked for {mode}, ran {used}")
            if rank_result is not None and not args.no_verify:
                same = bool(np.array_equal(rr.cpu().numpy(), rank_result[1].cpu().numpy())
                            and np.array_equal(rd.cpu().numpy().view(np.uint32),
                                               rank_result[0].cpu().numpy().view(np.uint32)))
                assert same, f"serve leg ({mode}) differs from the one-process-per-GPU result"
                rec["equals_rank_path"] = same
            out["gathers"][mode] = rec
    finally:
        if old is None:
            os.environ.pop("FENIX_AMD_GATHER", None)
        else:
            os.environ["FENIX_AMD_GATHER"] = old
    return out


def batch_leg(eng, shard, image, img_bytes, n, d, k, args, nb=256, mname="cosine"):
    """BASELINE configs[2] on the bench's resident shard and filter image: a
    256-query cosine batch (query seed 2), W warmup + K timed searches, HIP
    events around each search's launches; three of its queries checked bit
    for bit against the exact per-query scan."""
    from fenix_amd import _lib

    dev = shard.data.device
    mb = _lib.METRICS[mname]
    qb = torch.empty((nb, d), dtype=torch.float32, device=dev)
    eng.fill(qb, seed=2)
    bd = torch.empty((nb, k), dtype=torch.float32, device=dev)
    br = torch.empty((nb, k), dtype=torch.int64, device=dev)

    def one(ev=None):
        if ev is not None:
            ev[0].record()
        st = eng.scan(shard, qb, mb, k)
        eng.reduce(shard, qb, mb, k, st, bd, br)
        if ev is not None:
            ev[1].record()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    for _ in range(args.warmup):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        one(ev[i])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    span = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    same = None
    if not args.no_verify:
        idx = [0, 1, nb - 1]
        sub = qb[idx].contiguous()
        sd = torch.empty((len(idx), k), dtype=torch.float32, device=dev)
        sr = torch.empty((len(idx), k), dtype=torch.int64, device=dev)
        with _lib.options(batched=0, single_query_image=0):
            st = eng.scan(shard, sub, mb, k)
            eng.reduce(shard, sub, mb, k, st, sd, sr)
        same = bool(np.array_equal(sr.cpu().numpy(), br[idx].cpu().numpy()) and np.array_equal(
            sd.cpu().numpy().view(np.uint32), bd[idx].cpu().numpy().view(np.uint32)))
        assert same, "configs[2] batch differs from the exact scan"
    pass_bytes = img_bytes + nb * d * 4
    # HBM bytes per search from the SHA-matched counter pass of the same
    # workload (bench.py --nq 256 --metric cosine, tools/round_end.sh)
    traffic = pmc_traffic(f"{n}x{d}_f32_{mname}_k{k}_q{nb}", "filter_img", _lib.library_sha())
    return {
        "workload": f"{n}x{d} f32 {mname} kNN k={k}, {nb}-query batch (query seed 2), "
                    "same shard and filter image",
        "ms_per_step": el * 1e3 / args.steps,
        "vectors_per_s": n * nb * args.steps / el,
        "kernel_ms": span,
        "kernel": "filter phases (int8 MFMA bound filter) + thresholds + rescoring + select",
        "bytes_per_search": pass_bytes,
        "achieved_gbs_over_image": pass_bytes / (span * 1e-3) / 1e9,
        "frac_over_image": check_frac("configs2.frac_over_image",
                                      pass_bytes / (span * 1e-3) / 1e9 / HBM_PEAK_GBS),
        "mfma_tops": 2.0 * n * nb * d / (span * 1e-3) / 1e12,   # int8 ops, not flops
        "mfma_peak_tops": MFMA_F16_PEAK_TFS * 2,
        "traffic": traffic,
        "traffic_over_image": (traffic / pass_bytes) if traffic else None,
        "sample_bit_identical": same,
    }


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


if __name__ == "__main__":
    main()
