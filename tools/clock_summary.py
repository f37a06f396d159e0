"""Effective clock per recon kernel from tools/profile_clock.sh output (dev tool)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    if "recon" not in r["Kernel_Name"]:
        continue
    k = r["Kernel_Name"].split("(")[0].split("::")[-1]
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    agg[k]["dur"].append(dur)
for k, v in agg.items():
    g = sum(v["GRBM_GUI_ACTIVE"]) / len(v["GRBM_GUI_ACTIVE"])
    t = sum(v["dur"]) / len(v["dur"])
    print(f"{k:28s} GUI_ACTIVE {g:12.0f}  dur {t * 1e3:7.4f} ms  clock {g / t / 1e9:5.2f} GHz")
