"""Summarise a tools/profile.sh run (gpurun_out/prof_<tag>/) for the recon kernel.

    python tools/prof_summary.py <tag> [--mbs-per-launch-total N] [--out profiles/<file>.md]

Prints the rocprofv3 kernel stats, per-dispatch averages of every PMC counter, and the HBM
traffic per dispatch derived the way MI355X_MICROARCH.md prescribes (FETCH_SIZE/WRITE_SIZE are
KiB; gfx950 FETCH_SIZE under-reports wide streaming reads by 2x, so both the raw and the x2
value are shown).
"""
import argparse
import collections
import csv
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_counters(d, name):
    path = os.path.join(d, name, f"{name}_counter_collection.csv")
    if not os.path.exists(path):
        return {}
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if "recon_kernel" not in r["Kernel_Name"]:
            continue
        per[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--out")
    ap.add_argument("--json", help="write HBM traffic per bench step (bytes) for bench.py's roofline.traffic")
    ap.add_argument("--steps-total", type=int, default=18,
                    help="batches the profiled bench run decodes: steps + warmup + the 6 batches of its one-stream "
                         "per-kernel context (bench.py: 10 + 2 + 6 by default)")
    ap.add_argument("--config", default="c2")
    ap.add_argument("--gops", type=int, default=64)
    args = ap.parse_args()
    d = os.path.join(REPO, "gpurun_out", f"prof_{args.tag}")
    lines = [f"# rocprofv3 summary: {args.tag}", ""]
    stats = os.path.join(d, "ktrace", "ktrace_kernel_stats.csv")
    if os.path.exists(stats):
        lines.append("## kernel stats (rocprofv3 --kernel-trace --stats)")
        lines.append("")
        lines.append("| kernel | calls | avg ns | total ns | % |")
        lines.append("|---|---|---|---|---|")
        for r in csv.DictReader(open(stats)):
            lines.append(f"| {r['Name'][:70]} | {r['Calls']} | {float(r['AverageNs']):.0f} | "
                         f"{float(r['TotalDurationNs']):.0f} | {float(r['Percentage']):.2f} |")
        lines.append("")
    trace = os.path.join(d, "ktrace", "ktrace_kernel_trace.csv")
    durs = []
    if os.path.exists(trace):
        for r in csv.DictReader(open(trace)):
            if "recon_kernel" in r["Kernel_Name"]:
                durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    counters = {}
    for name in ("fetch", "write", "sq1", "sq2", "tcc"):
        counters.update(load_counters(d, name))
    if counters:
        lines.append("## PMC counters, recon_kernel, mean per dispatch")
        lines.append("")
        lines.append("| counter | mean per dispatch | dispatches |")
        lines.append("|---|---|---|")
        for k in sorted(counters):
            v = counters[k]
            lines.append(f"| {k} | {statistics.mean(v):.4g} | {len(v)} |")
        lines.append("")
        if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
            f = statistics.mean(counters["FETCH_SIZE"]) * 1024
            w = statistics.mean(counters["WRITE_SIZE"]) * 1024
            lines.append(f"HBM-side bytes per dispatch: FETCH {f / 1e6:.1f} MB raw ({2 * f / 1e6:.1f} MB with the "
                         f"gfx950 x2 correction), WRITE {w / 1e6:.1f} MB; traffic (FETCH x2 + WRITE) "
                         f"{(2 * f + w) / 1e6:.1f} MB")
            if durs:
                lines.append(f"kernel-trace mean duration {statistics.mean(durs) / 1e3:.1f} us over {len(durs)} dispatches")
            fsum = sum(counters["FETCH_SIZE"]) * 1024 * 2 / args.steps_total
            wsum = sum(counters["WRITE_SIZE"]) * 1024 / args.steps_total
            lines.append(f"per bench step ({args.steps_total} steps profiled): FETCH x2 {fsum / 1e9:.3f} GB + WRITE "
                         f"{wsum / 1e9:.3f} GB = {(fsum + wsum) / 1e9:.3f} GB")
            reqs = None
            if "TCC_HIT_sum" in counters and "TCC_MISS_sum" in counters:
                hit = sum(counters["TCC_HIT_sum"]) / args.steps_total
                miss = sum(counters["TCC_MISS_sum"]) / args.steps_total
                reqs = hit + miss
                lines.append(f"L2 (TCC) requests per bench step: {reqs / 1e6:.1f} M (hit rate {hit / reqs:.3f})")
            if args.json:
                import json
                out = {"tag": args.tag, "config": args.config, "gops": args.gops,
                       "traffic_bytes_per_step": int(fsum + wsum), "fetch_x2_bytes_per_step": int(fsum),
                       "fetch_raw_bytes_per_step": int(fsum / 2), "write_bytes_per_step": int(wsum),
                       "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (KiB), summed over the "
                                 "recon_kernel dispatches of the profiled bench run / steps. FETCH_SIZE = 64 B per "
                                 "L2-to-fabric read request (tools/fetch_calib.hip: a coalesced 128-B line is one "
                                 "request, and so is a 20-B tap row on one missed line), so raw FETCH is the lower "
                                 "bound of the bytes read and FETCH x2 (128 B per request, the gfx950 correction of "
                                 "MI355X_MICROARCH.md) the upper; traffic = FETCH x2 + WRITE (WRITE_SIZE is exact "
                                 "for the kernel's 64-B and 128-B row stores)"}
                if reqs is not None:
                    out.update({"l2_requests_per_step": int(reqs), "l2_hit_rate": round(hit / reqs, 4),
                                "l2_request_method": "TCC_HIT_sum + TCC_MISS_sum (one request per 128-B line an "
                                                     "L1 miss touches, tools/fetch_calib.hip)"})
                with open(args.json, "w") as fh:
                    json.dump(out, fh, indent=1)
        lines.append("")
    text = "\n".join(lines)
    print(text)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    sys.exit(main())
