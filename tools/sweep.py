"""Same-box sweep / A/B driver over bench.py (replaces the one-off ab_*.sh).

    python tools/sweep.py [--libs new,old] [--reps 2] [--steps 10] [--warmup 2]
                          [--out gpurun_out/sweep.jsonl] -- "ARGS1" "ARGS2" ...

Each quoted ARGS is one bench.py configuration (leading NAME=VALUE tokens are
environment variables for that run, e.g. "FX_FILTER_DIAG=2 --nq 256" with
``--libs diag`` for the diagnostic build's switches); every (rep, config, lib) runs
bench.py in its own process under a time limit (``--no-cpu-baseline`` added),
and one line per run is printed and appended to ``--out``.  A library NAME
other than ``new`` is ``fenix_amd/lib/libfenix_knn_NAME.so`` (loaded through
FENIX_AMD_LIB; build it first, e.g. ``make -C fenix_amd/csrc
BUILD=build_old OUT=../lib/libfenix_knn_old.so``).  Box-to-box HBM variance
is a few per cent, larger than most kernel changes: compare within one call.
The first failing run ends the sweep with its exit status.
"""

from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def summary(rec: dict) -> dict:
    out = {"ms": round(rec["ms_per_step"], 4), "kernel_ms": round(rec["roofline"]["kernel_ms"], 4),
           "frac": round(rec["roofline"]["frac"], 4)}
    acc = rec.get("accelerated_exact")
    if acc:
        out.update(acc_ms=round(acc["ms_per_step"], 4), acc_kernel_ms=round(acc["kernel_ms"], 4),
                   acc_same=acc["bit_identical"])
    return out


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--libs", default="new")
    p.add_argument("--reps", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--timeout", type=int, default=240)
    p.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sweep.jsonl"))
    p.add_argument("configs", nargs="+")
    a = p.parse_args()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    for rep in range(a.reps):
        for cfg in a.configs:
            for lib in a.libs.split(","):
                env = dict(os.environ)
                env.pop("FENIX_AMD_LIB", None)
                if lib != "new":
                    env["FENIX_AMD_LIB"] = os.path.join(ROOT, "fenix_amd", "lib",
                                                        f"libfenix_knn_{lib}.so")
                toks = shlex.split(cfg)
                while toks and "=" in toks[0] and toks[0].split("=", 1)[0].isupper():
                    key, val = toks.pop(0).split("=", 1)
                    env[key] = val
                cmd = ["timeout", "-k", "10", str(a.timeout), sys.executable, "-u",
                       os.path.join(ROOT, "bench.py"), *toks, "--steps",
                       str(a.steps), "--warmup", str(a.warmup), "--no-cpu-baseline"]
                r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT, env=env)
                if r.returncode != 0:
                    print(f"FAILED rc={r.returncode} lib={lib} args={cfg}\n{r.stderr[-3000:]}",
                          flush=True)
                    return r.returncode
                rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
                line = {"rep": rep, "lib": lib, "args": cfg, **summary(rec)}
                print(json.dumps(line), flush=True)
                with open(a.out, "a") as f:
                    f.write(json.dumps({**line, "record": rec}) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
