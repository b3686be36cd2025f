"""One warm io.index.call on a single clock: HIP API calls (host), kernels and
memory copies (device) from a rocprofv3 --runtime-trace --kernel-trace
--memory-copy-trace run of tools/profile_call.py, relative to the search's
first HIP call.  Shows where the host part of a served search goes: the
host time before the first kernel starts, the device span, and the tail
from the last kernel to the return of the synchronisation.

    python tools/host_gap.py gpurun_out/r06/rtrace/run [--search 15] [--anchor qprep8]
"""

from __future__ import annotations

import argparse
import csv
import os


def rows(path: str):
    if not os.path.exists(path):
        return []
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("prefix", help="rocprofv3 -d DIR -o NAME: DIR/NAME")
    p.add_argument("--search", type=int, default=15, help="which anchored search (0-based)")
    p.add_argument("--anchor", default="qprep8", help="kernel-name substring of a search's first kernel")
    a = p.parse_args()
    ev = []
    for r in rows(a.prefix + "_kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:70]))
    for r in rows(a.prefix + "_hip_api_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "H", r["Function"]))
    for r in rows(a.prefix + "_memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "M",
                   f'{r.get("Direction", "")} {r.get("Bytes", "")}B'))
    ev.sort()
    anchors = [e for e in ev if e[2] == "K" and a.anchor in e[3]]
    if len(anchors) <= a.search + 1:
        raise SystemExit(f"only {len(anchors)} searches anchored on {a.anchor!r}")
    k0, k1 = anchors[a.search][0], anchors[a.search + 1][0]
    # the search's host part starts after the previous search's last synchronisation
    syncs = [e for e in ev if e[2] == "H" and "Synchronize" in e[3] and e[1] < k0]
    t0 = syncs[-1][1] if syncs else k0
    win = [e for e in ev if t0 <= e[0] < k1]
    first_api = min((e[0] for e in win if e[2] == "H"), default=t0)
    for s, e, kind, name in win:
        if kind == "H" and e - s < 2000 and "Synchronize" not in name:
            continue  # (sub-2 us API calls: counted below, not listed)
        print(f"{(s - first_api) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {kind} {name}")
    nh = sum(1 for e in win if e[2] == "H")
    kern = [e for e in win if e[2] == "K"]
    last_sync = [e for e in win if e[2] == "H" and "Synchronize" in e[3]]
    print(f"HIP calls {nh}; first HIP call -> first kernel start "
          f"{(kern[0][0] - first_api) / 1e3:.1f} us; kernels span "
          f"{(kern[-1][1] - kern[0][0]) / 1e3:.1f} us")
    if last_sync:
        print(f"last kernel end -> synchronisation returns {(last_sync[-1][1] - kern[-1][1]) / 1e3:.1f} us; "
              f"first HIP call -> sync returns {(last_sync[-1][1] - first_api) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
