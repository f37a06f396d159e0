"""Summary of a tools/pmc5.sh run: per recon kernel, the rocprofv3 kernel-trace mean and every
PMC counter per dispatch, plus derived rates (dev tool).

    python tools/pmc5_summary.py gpurun_out/pmc5_<tag>

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports
half the bytes of wide coalesced streaming reads, so the table shows FETCH raw and x2 (the bound
pair for a mix of streaming and gathered reads).
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def kname(n):
    m = re.search(r"recon_kernel<(\d), (\d), 0>", n)
    return f"<{m.group(1)},{m.group(2)},0>" if m else None


def main(d):
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k:
                rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    # per-kernel durations from the kernel trace, the timed batches only (without onestream.py's
    # warm-up batch and the placement calibration in it): the launches its HIP-event table averages
    stats = {}
    for f in glob.glob(os.path.join(d, "ktrace", "*kernel_trace.csv")):
        disp = sorted((int(r["Correlation_Id"]), kname(r["Kernel_Name"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                      for r in csv.DictReader(open(f)) if kname(r["Kernel_Name"]))
        ev0 = None
        for line in open(os.path.join(d, "ktrace.log")) if os.path.exists(os.path.join(d, "ktrace.log")) else []:
            if line.startswith("{"):
                ev0 = json.loads(line)
        nl = sum(v["launches_per_batch"] for v in ev0["per_kernel"].values()) if ev0 else 5
        reps = ev0["batches_decoded"] - 1 if ev0 else len(disp) // nl - 1
        timed = disp[-reps * nl:]  # the timed batches are the last ones (placement calibration batches come first)
        by = collections.defaultdict(list)
        for _, k, ns in timed:
            by[k].append(ns / 1e6)
        for k, v in by.items():
            stats[k] = (len(v), sum(v) / len(v), min(v), max(v))
    ev = None
    log = os.path.join(d, "ktrace.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{"):
                ev = json.loads(line)
    print(f"# rocprofv3, one-stream bench batch ({os.path.basename(d)})\n")
    if ev:
        print(f"config {ev['config']}, {ev['gops']} GOPs, {ev['frames']} frames per batch, parity {ev['parity']}, "
              f"one-stream batch span {ev['span_ms']} ms (HIP events)\n")
    print("| kernel | mode | timed dispatches | rocprof mean ms (min / max) | HIP-event mean ms | rocprof / events | algorithmic bytes | frac (rocprof mean) |")
    print("|---|---|---|---|---|---|---|---|")
    for k in sorted(stats):
        calls, avg, mn, mx = stats[k]
        e = None
        if ev:
            e = next((v for n, v in ev["per_kernel"].items() if n.replace(" ", "").replace("recon_kernel", "") == k), None)
        ab = e["algorithmic_bytes_per_launch"] if e else None
        frac = f"{ab / (avg / 1e3) / 8.0e12:.4f}" if ab else "-"
        ratio = f"{avg / e['avg_launch_ms']:.3f}" if e else "-"
        print(f"| `recon_kernel{k}` | {e['mode'] if e else '-'} | {calls} | {avg:.4f} ({mn:.4f} / {mx:.4f}) | "
              f"{e['avg_launch_ms'] if e else '-'} | {ratio} | {ab} | {frac} |")
    print()
    for k in sorted(rows):
        c = {n: sum(v) / len(v) for n, v in rows[k].items()}
        print(f"## `recon_kernel{k}` (mean per dispatch)\n")
        for n in sorted(c):
            print(f"- {n}: {c[n]:,.1f}")
        der = []
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            f, w = c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
            der.append(f"HBM-side bytes: FETCH raw {f / 1e9:.3f} GB, x2 {2 * f / 1e9:.3f} GB; WRITE {w / 1e9:.3f} GB")
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            der.append(f"L2 hit rate {c['TCC_HIT_sum'] / max(1.0, c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.3f}")
        if "TCP_TCC_READ_REQ_sum" in c and "TCP_TCC_READ_REQ_LATENCY_sum" in c:
            der.append(f"L1->L2 read latency {c['TCP_TCC_READ_REQ_LATENCY_sum'] / max(1.0, c['TCP_TCC_READ_REQ_sum']):.0f} cycles "
                       f"over {c['TCP_TCC_READ_REQ_sum'] / 1e6:.2f} M requests")
        if "TCP_TCC_WRITE_REQ_sum" in c and "TCP_TCC_WRITE_REQ_LATENCY_sum" in c:
            der.append(f"L1->L2 write latency {c['TCP_TCC_WRITE_REQ_LATENCY_sum'] / max(1.0, c['TCP_TCC_WRITE_REQ_sum']):.0f} cycles "
                       f"over {c['TCP_TCC_WRITE_REQ_sum'] / 1e6:.2f} M requests")
        if "TCP_UTCL1_TRANSLATION_MISS_sum" in c and "TCP_UTCL1_TRANSLATION_HIT_sum" in c:
            t = c["TCP_UTCL1_TRANSLATION_MISS_sum"] + c["TCP_UTCL1_TRANSLATION_HIT_sum"]
            der.append(f"UTCL1 translation miss rate {c['TCP_UTCL1_TRANSLATION_MISS_sum'] / max(1.0, t):.4f}")
        if der:
            print("\nderived: " + "; ".join(der))
        print()


if __name__ == "__main__":
    main(sys.argv[1])
