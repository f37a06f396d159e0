"""Mean counter value per recon kernel over every pass under a profile directory (dev tool)."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "recon" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("(")[0].split("recon_kernel")[-1]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[k]["dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
for k in sorted(agg):
    print(k)
    for c, v in sorted(agg[k].items()):
        print(f"   {c:34s} {sum(v) / len(v):16.1f}")
