"""Copy a gpurun profile run into profiles/ (tracked): kernel-trace stats,
PMC summary, and per-launch HBM traffic of each kernel (gfx950 correction:
FETCH_SIZE reports half the bytes of 16-B/lane streaming reads, so it is
doubled; WRITE_SIZE is exact for 16-B/lane stores — MI355X_MICROARCH.md §HBM).

    python scripts/make_profile_summary.py gpurun_out/prof_r1 r1
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "bench_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
summ = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "pmc_summary.py"), src],
                      capture_output=True, text=True).stdout
open(os.path.join(dst, f"{tag}_pmc_summary.txt"), "w").write(summ)
agg = defaultdict(lambda: defaultdict(list))
for path in sorted(glob.glob(f"{src}/pmc*/p_counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        agg[(r["Kernel_Name"], int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if "End_Timestamp" in r and "Start_Timestamp" in r and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            agg[(r["Kernel_Name"], int(r["Grid_Size"]))]["_dur_ns"].append(
                float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
traffic = {}
for (name, grid), d in agg.items():
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        f = 2.0 * 1024 * sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
        w = 1024.0 * sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
        traffic[f"{name}|{grid}"] = {"fetch_bytes": f, "write_bytes": w, "hbm_bytes": f + w,
                                     "mfma_busy_cycles": (sum(d["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(d["SQ_VALU_MFMA_BUSY_CYCLES"])
                                                          if "SQ_VALU_MFMA_BUSY_CYCLES" in d else None),
                                     "grbm_gui_active": (sum(d["GRBM_GUI_ACTIVE"]) / len(d["GRBM_GUI_ACTIVE"])
                                                         if "GRBM_GUI_ACTIVE" in d else None),
                                     "pmc_dur_ns": (sum(d["_dur_ns"]) / len(d["_dur_ns"]) if d.get("_dur_ns") else None)}
        t = traffic[f"{name}|{grid}"]
        if t["mfma_busy_cycles"] is not None and t["grbm_gui_active"]:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; SQ_VALU_MFMA_BUSY_CYCLES over the 1024 SIMDs
            t["mfma_util"] = t["mfma_busy_cycles"] / (t["grbm_gui_active"] / 8 * 1024)
            if t["pmc_dur_ns"]:
                t["clock_ghz"] = t["grbm_gui_active"] / 8 / t["pmc_dur_ns"]
json.dump(traffic, open(os.path.join(dst, f"{tag}_traffic.json"), "w"), indent=1)
log = os.path.join(src, "trace.log")
if os.path.exists(log):
    for line in open(log):
        if line.startswith("{"):
            open(os.path.join(dst, f"{tag}_bench_under_rocprof.json"), "w").write(line)
print("wrote", dst)
