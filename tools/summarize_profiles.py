"""Turn rocprofv3 CSV output (gpurun_out/) into the committed profiles/ files.

    python tools/summarize_profiles.py --round 1 --stats gpurun_out/prof/run_kernel_stats.csv \
        --pmc gpurun_out/pmc/run_counter_collection.csv --workload 10000000x768_f32_l2_k100_q1 \
        --algo-bytes 30720003072

* copies the --kernel-trace --stats summary to profiles/rNN_kernel_stats.csv;
* writes profiles/rNN_pmc_<workload>.json: FETCH_SIZE per launch of the scan
  kernel, converted to bytes with the two gfx950 corrections of
  MI355X_MICROARCH.md §HBM (FETCH_SIZE is in KiB; it reports exactly half of
  the bytes of a wide coalesced streaming read, so x2).  bench.py reads
  ``hbm_bytes_per_launch`` from it for roofline.traffic, only when its
  ``library_sha`` equals the loaded library's (a kernel change makes a pass
  stale).  ``--kernel`` is a substring; with ``--per-search N`` every N
  matching launches (the phases of one batched search) are summed.
"""

from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--round", type=int, required=True)
    p.add_argument("--stats")
    p.add_argument("--pmc")
    p.add_argument("--workload", required=True)
    p.add_argument("--algo-bytes", type=float, required=True)
    p.add_argument("--kernel", default="fx::scan_kernel")
    p.add_argument("--tag", default="")
    p.add_argument("--per-search", type=int, default=1,
                   help="matching launches per search (summed): the filter's phases")
    p.add_argument("--searches", type=int, default=0,
                   help="searches the run made: FETCH_SIZE of every matching launch summed "
                        "and divided by it (instead of --per-search)")
    p.add_argument("--library-sha", default=None,
                   help="SHA-256 prefix of the library the pass ran (default: hash the "
                        "in-tree fenix_amd/lib/libfenix_knn.so, which must be that build)")
    p.add_argument("--source-cmd", default="")
    a = p.parse_args()
    out_dir = os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    pre = f"r{a.round:02d}{a.tag}"
    if a.stats:
        shutil.copy(a.stats, os.path.join(out_dir, f"{pre}_kernel_stats.csv"))
        # the named kernel's average launch, from the same summary
        for r in csv.DictReader(open(a.stats)):
            if a.kernel in r.get("Name", r.get("KernelName", "")):
                print(json.dumps({"kernel": r.get("Name"), "calls": r.get("Calls"),
                                  "average_ns": r.get("AverageNs")}))
    if a.pmc:
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(a.pmc)):
            if a.kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        fetch = vals.get("FETCH_SIZE", [])
        if a.searches:
            searches = a.searches
            mean_kib = sum(fetch) / searches
            a.per_search = len(fetch) / searches
        else:
            searches = len(fetch) // a.per_search
            mean_kib = sum(fetch[: searches * a.per_search]) / searches
        hbm = mean_kib * 1024 * 2
        if a.library_sha is None:
            import sys

            sys.path.insert(0, ROOT)
            from fenix_amd import _lib

            a.library_sha = _lib.library_sha()
        rec = {
            "workload": a.workload,
            "kernel": a.kernel,
            "library_sha": a.library_sha,
            "launches": len(fetch),
            "launches_per_search": a.per_search,
            "FETCH_SIZE_kib_per_launch": mean_kib,
            "hbm_bytes_per_launch": hbm,
            "algorithmic_bytes_per_launch": a.algo_bytes,
            "traffic_over_algorithmic": hbm / a.algo_bytes,
            "correction": "FETCH_SIZE is KiB; x2 because gfx950 reports half the bytes of a "
                          "16-B/lane coalesced stream (MI355X_MICROARCH.md, HBM section)",
            "source": os.path.relpath(a.pmc, ROOT),
            "command": a.source_cmd,
        }
        with open(os.path.join(out_dir, f"{pre}_pmc_{a.workload}.json"), "w") as f:
            json.dump(rec, f, indent=1)
        print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
