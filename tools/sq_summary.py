"""Summarise one rocprofv3 SQ counter pass (tools/pmc.sh) for the longest
launch of a kernel: the counters, and the derived shares of
tools/../profiles/r01_filter_pmc_sq.txt (SQ_WAVE_CYCLES, SQ_WAIT_* and
SQ_ACTIVE_* count quad-cycles).

    python tools/sq_summary.py gpurun_out/pmc_NAME/run_counter_collection.csv KERNEL_SUBSTRING
"""
import collections
import csv
import sys

path, kern = sys.argv[1], sys.argv[2]
by = collections.defaultdict(dict)
names = {}
for r in csv.DictReader(open(path)):
    if kern not in r["Kernel_Name"]:
        continue
    did = r["Dispatch_Id"]
    by[did][r["Counter_Name"]] = by[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    names[did] = r["Kernel_Name"]
# the dispatch with the most wave cycles: the final pass
did = max(by, key=lambda k: by[k].get("SQ_WAVE_CYCLES", 0.0))
c = by[did]
print(f"# {names[did][:90]}  (dispatch {did}, {len(by)} matching dispatches)")
for k in sorted(c):
    print(f"{k:28s} {c[k]:.4g}")
wc = c.get("SQ_WAVE_CYCLES", 0.0)
if wc:
    wait = c.get("SQ_WAIT_ANY", 0.0)
    act = c.get("SQ_ACTIVE_INST_ANY", 0.0)
    print("# derived:")
    print(f"waves parked in s_waitcnt / barrier  {100 * wait / wc:.1f}%")
    print(f"waves issuing                        {100 * act / wc:.1f}%")
    print(f"waves issue-stalled                  {100 * (wc - wait - act) / wc:.1f}%  "
          f"(of which LDS issue {100 * c.get('SQ_WAIT_INST_LDS', 0.0) / wc:.1f}%)")
g = c.get("GRBM_GUI_ACTIVE", 0.0)
if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
    print(f"MFMA busy / SIMD cycles              {100 * c['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * g / 8):.1f}%"
          "  (1024 SIMDs x GRBM_GUI_ACTIVE/8)")
