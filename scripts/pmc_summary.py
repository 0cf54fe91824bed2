"""Summarise rocprofv3 --pmc CSVs: per (kernel, grid) mean counter values."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
agg = defaultdict(lambda: defaultdict(list))
for path in sorted(glob.glob(f"{root}/pmc*/p_counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        key = (r["Kernel_Name"][:70], int(r["Grid_Size"]))
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[key]["_dur_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
for key, d in sorted(agg.items(), key=lambda kv: -sum(kv[1]["_dur_ns"])):
    print(key)
    for c, v in sorted(d.items()):
        print(f"    {c:34s} {sum(v) / len(v):16.1f}  (n={len(v)})")
