"""bench.py keeps the driver's output contract (one JSON line with metric,
value, roofline, cpu_baseline ...) on small shapes of each path it reports:
the single-query scan, the batched filter, fp16 rows and quint8 codes."""

from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
        "roofline", "cpu_baseline"}


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_bench(*args: str, env=None) -> dict:
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                         capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("extra", [
    ("--d", "768"),
    ("--nq", "16", "--metric", "cosine"),
    ("--dtype", "f16", "--d", "1536", "--k", "1000", "--metric", "inner_product"),
    ("--dtype", "qu8"),
])
def test_bench_contract(extra):
    rec = run_bench("--rows", "300000", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                    *extra)
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == 1 and rec["steps"] == 3 and rec["value"] > 0
    roof = rec["roofline"]
    assert roof["bound"] in ("hbm", "mfma") and roof["peak"] > 0
    assert roof["frac"] == pytest.approx(roof["achieved"] / roof["peak"])
    assert rec["config"]["rows_per_gpu"] == 300000


def test_bench_cpu_baseline_fields():
    rec = run_bench("--rows", "200000", "--steps", "2", "--warmup", "1", "--cpu-rows", "20000",
                    "--cpu-seconds", "0.5")
    cpu = rec["cpu_baseline"]
    assert cpu["kind"] in ("port", "reference") and cpu["cores"] >= 1 and cpu["value"] > 0


def test_bench_rccl_path_one_rank():
    """The N > 1 path of bench.py (RCCL process group, all-gather of the per-rank
    top-k, merge, barriers, max-over-ranks all-reduce) launched the way the
    driver launches it, with one rank: the one-GPU box runs every RCCL call
    the 8-GPU scaling run makes."""
    env = dict(os.environ, FENIX_AMD_BENCH_DIST="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--rows", "300000", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["config"]["parallelism"] == "row-shard x1, one process per GPU + RCCL all-gather"
    assert rec["n_gpus"] == 1 and rec["value"] > 0


def test_bench_gpus_n_launches_n_ranks():
    """`bench.py --gpus 2` without a launcher starts 2 ranks itself (here
    with gloo, two ranks sharing the one GPU of the box: RCCL refuses a
    duplicate device) and reports n_gpus 2 over 2 x rows, the strong-scaling
    leg (--rows in total, half per rank) and the single-process serve leg
    (rank 0 alone, two shards through engine._search_all, merged on the one
    device since the ordinal repeats), whose result bench.py checks against
    the ranks' merge.  rank 0 also times the CPU baseline after the timed
    legs while rank 1 waits on the store, so the N > 1 line carries one."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    rec = run_bench("--gpus", "2", "--dist-backend", "gloo", "--rows", "200000", "--steps", "3",
                    "--warmup", "1", "--cpu-rows", "20000", "--cpu-seconds", "0.5",
                    "--serve-devices", "0,0", env=env)
    assert rec["n_gpus"] == 2
    assert rec["config"]["total_rows"] == 400000
    assert rec["config"]["parallelism"].startswith(
        "row-shard x2, one process per GPU + gloo all-gather; strong leg: 200000 rows over 2")
    strong = rec["strong"]
    assert strong["total_rows"] == 200000 and strong["rows_per_gpu"] == 100000
    assert 0 < strong["frac"] <= 1
    serve = rec["serve"]
    assert "error" not in serve, serve
    assert list(serve["gathers"]) == ["none"]
    assert serve["gathers"]["none"]["equals_rank_path"] is True
    cpu = rec["cpu_baseline"]
    assert cpu is not None and cpu["kind"] == "port" and cpu["value"] > 0 and cpu["cores"] >= 1


def test_bench_serve_devices_one_rank():
    """--serve-devices on a single rank (no process group): one process, three
    row shards on the one GPU, merged there."""
    rec = run_bench("--rows", "200000", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                    "--no-accelerated", "--serve-devices", "0,0,0")
    serve = rec["serve"]
    assert serve["total_rows"] == 600000 and serve["gathers"]["none"]["value"] > 0


def test_bench_gpus_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--rows", "100000", "--steps", "1", "--no-cpu-baseline"],
                         capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert out.returncode != 0
    assert "WORLD_SIZE=1" in out.stderr
