"""Per-dispatch timeline of the last batched search in a rocprofv3 kernel trace.

    python tools/ktrace_summary.py gpurun_out/prof3/run_kernel_trace.csv > profiles/r01_filter_ktrace.txt

A batched search starts at its ``qprep_kernel``; everything from the last one
to the end of the trace is one search (bench.py's final timed step).  The sum
of the durations is what bench.py's ``roofline.kernel_ms`` brackets with HIP
events for the filter path.
"""

from __future__ import annotations

import csv
import sys


def main() -> None:
    path = sys.argv[1]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    first = max(i for i, r in enumerate(rows) if "qprep_kernel" in r["Kernel_Name"])
    last = rows[first:]
    # bench.py's cpu-side sanity check and exit follow the last search: keep
    # the dispatches of the search only (up to the last merge after rescoring)
    end = max(i for i, r in enumerate(last) if "merge_kernel" in r["Kernel_Name"])
    last = last[: end + 1]
    t0 = int(last[0]["Start_Timestamp"])
    print("# one 256-query cosine search over 10M x 768 f32 (bench.py --nq 256 --metric cosine),")
    print(f"# rocprofv3 --kernel-trace ({path}); start offset and duration in us")
    print(" start_us    dur_us  kernel")
    total = 0
    for r in last:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        total += e - s
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:9.1f}  {r['Kernel_Name'][:100]}")
    span = int(last[-1]["End_Timestamp"]) - t0
    print(f"# sum of kernel durations: {total / 1e3:.1f} us; first start to last end: {span / 1e3:.1f} us")


if __name__ == "__main__":
    main()
