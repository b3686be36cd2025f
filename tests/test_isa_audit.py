"""Compile-time audit of the MFMA kernels' result reads.

Every v_mfma result must be read at least 12 issue slots after the MFMA (the
8-pass XDL requirement, measured on gfx950 by tools/mfma_race.hip:
profiles/r05_mfma_race.jsonl), and every path from an accumulating kernel's
last MFMA to the epilogue's first read must cross a workgroup barrier: the
resident-slice kernel without one moved candidate counts between identical
runs, and neither 64 extra wait states nor draining its own loads fixed it
(profiles/r05_img6_race_variants*.log).  tools/mfma_hazard.py walks every
control-flow path of the hipcc -S listing."""

from __future__ import annotations

import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "fenix_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
SOURCES = ["knn_filter_q64i.hip", "knn_filter_q128.hip", "knn_filter.hip", "knn_code.hip"]


@pytest.fixture(scope="module")
def listings(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa")

    def one(src):
        dst = os.path.join(out, src.replace(".hip", ".s"))
        subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-DFX_NONTEMPORAL=1",
                        "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S",
                        "-o", dst, os.path.join(CSRC, src)],
                       check=True, capture_output=True, cwd=CSRC, timeout=600)
        return dst

    with ThreadPoolExecutor(len(SOURCES)) as ex:
        return dict(zip(SOURCES, ex.map(one, SOURCES)))


@pytest.mark.parametrize("src", SOURCES)
def test_mfma_results_read_late_and_behind_a_barrier(listings, src):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mfma_hazard.py"),
                          listings[src]], capture_output=True, text=True, check=True, timeout=600)
    recs = [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert recs, f"no MFMA kernel found in {src}"
    for r in recs:
        assert r["min_states"] >= 12, r
        assert r["min_states_no_barrier"] is None, r
