"""Per-kernel dynamic VALU / LDS instruction counts and durations per ablation (dev tool)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
for a in ["0", "1", "2", "4", "32", "64"]:
    fs = glob.glob(f"{d}/a{a}/**/*counter_collection.csv", recursive=True)
    if not fs:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(fs[0])):
        if "recon" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("(")[0].split("recon_kernel")[-1]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[k]["dur"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    out = []
    for k in sorted(agg):
        v = agg[k]
        mean = lambda x: sum(x) / len(x)
        out.append(f"{k} valu {mean(v['SQ_INSTS_VALU']) / 1e6:7.1f}M lds {mean(v['SQ_INSTS_LDS']) / 1e6:5.1f}M "
                   f"{mean(v['dur']):.4f}ms")
    print(f"abl={a:3s} " + " | ".join(out))
