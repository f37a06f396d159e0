"""Step accounting from a rocprofv3 kernel trace of bench.py (dev tool): where a step's time goes
beyond its level launches.

    python tools/ktrace_gaps.py <kernel_trace.csv> [--sets 2] [--launches 5] [--skip 2] [--steps 10]

bench.py's timed region enqueues `steps` batches back to back after `skip` warm-up batches; each
batch is `launches` level launches per picture set, one stream per set (runtime.cpp
mp2vg_batch_decode).  The trace's recon dispatches are grouped per stream in issue order, batch b
of a stream = its dispatches [b * launches, (b + 1) * launches).  Per timed batch:

  * chain_ms   -- per set: the sum of its launch durations (the set's critical path if it ran alone)
  * gaps_ms    -- per set: idle time between its consecutive launches (end -> next start, same stream)
  * span_ms    -- first start to last end over every set of the batch
  * busy_ms    -- union of all the batch's launch intervals (time with at least one launch running)
  * idle_ms    -- span - busy: no recon launch running at all

and the whole timed region: wall (first start -> last end) / steps, against max(chain) per step.
Prints a markdown table and a JSON line.
"""
import argparse
import csv
import json
import sys
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--sets", type=int, default=2)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--skip", type=int, default=2, help="warm-up batches before the timed ones")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    per_stream = defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        if "recon_kernel" not in r["Kernel_Name"]:
            continue
        per_stream[int(r["Stream_Id"])].append((int(r["Correlation_Id"]), int(r["Start_Timestamp"]),
                                                int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    # the timed batches' sets: the streams with the most recon dispatches (the bench context's set
    # streams; the one-stream per-kernel context after the timed region adds its own stream)
    streams = sorted(per_stream, key=lambda s: -len(per_stream[s]))[:a.sets]
    for s in streams:
        per_stream[s].sort()
    rows = []
    for b in range(a.skip, a.skip + a.steps):
        chains, gaps, ivals = [], [], []
        for s in streams:
            d = per_stream[s][b * a.launches:(b + 1) * a.launches]
            if len(d) < a.launches:
                sys.exit(f"stream {s}: only {len(per_stream[s])} recon dispatches")
            chains.append(sum(e - st for _, st, e, _ in d) / 1e6)
            gaps.append(sum(d[i + 1][1] - d[i][2] for i in range(len(d) - 1)) / 1e6)
            ivals += [(st, e) for _, st, e, _ in d]
        ivals.sort()
        busy, cur_s, cur_e = 0, None, None
        for st, e in ivals:
            if cur_e is None or st > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = st, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        span = (max(e for _, e in ivals) - min(st for st, _ in ivals)) / 1e6
        rows.append({"batch": b, "chain_ms": [round(x, 4) for x in chains], "gaps_ms": [round(x, 4) for x in gaps],
                     "span_ms": round(span, 4), "busy_ms": round(busy / 1e6, 4), "idle_ms": round(span - busy / 1e6, 4)})
    first = min(per_stream[s][a.skip * a.launches][1] for s in streams)
    last = max(per_stream[s][(a.skip + a.steps) * a.launches - 1][2] for s in streams)
    wall_step = (last - first) / 1e6 / a.steps
    crit = sum(max(r["chain_ms"]) for r in rows) / len(rows)
    print("| batch | set chains (sum of launches) ms | set gaps ms | batch span ms | busy ms | idle ms |")
    print("|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['batch']} | {' / '.join(map(str, r['chain_ms']))} | {' / '.join(map(str, r['gaps_ms']))} | "
              f"{r['span_ms']} | {r['busy_ms']} | {r['idle_ms']} |")
    out = {"streams": streams, "timed_steps": a.steps, "wall_ms_per_step": round(wall_step, 4),
           "critical_chain_ms_per_step": round(crit, 4), "wall_over_critical": round(wall_step / crit, 4),
           "mean_set_gaps_ms": round(sum(sum(r["gaps_ms"]) for r in rows) / len(rows) / len(streams), 4),
           "mean_idle_ms": round(sum(r["idle_ms"] for r in rows) / len(rows), 4)}
    print()
    print(f"wall per step {out['wall_ms_per_step']} ms; longest set chain per step {out['critical_chain_ms_per_step']} ms "
          f"(wall / chain {out['wall_over_critical']}); per set {out['mean_set_gaps_ms']} ms of gaps between its "
          f"launches; {out['mean_idle_ms']} ms per batch with no launch running")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
