"""Per-kernel timeline of the last search in a rocprofv3 kernel trace (csv):
kernels from the last launch whose name contains MARK to the end."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
mark = sys.argv[2] if len(sys.argv) > 2 else "qprep"
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
start = idx[-1] if idx else 0
t0 = int(rows[start]["Start_Timestamp"])
busy = 0
for r in rows[start:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:9.1f}  {r['Kernel_Name'][:80]}  "
          f"grid={r.get('Grid_Size_X', '')}x{r.get('Grid_Size_Y', '')}")
print(f"kernel time {busy / 1000:.1f} us")
