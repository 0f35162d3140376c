"""Summarise a rocprofv3 kernel trace (CSV) per kernel and per launching host thread (= rank of
the in-process group): launches, total / average ns, and the union of busy GPU time, so that a
multi-rank run can be itemised against a one-rank run of the same subdomain size.

    python tools/kernel_trace_summary.py TRACE.csv [--its N] [--skip-first-solve]
"""
import argparse
import collections
import csv
import json
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--its", type=int, default=0, help="CG iterations per solve (per-iteration figures)")
ap.add_argument("--solves", type=int, default=2, help="solves per rank in the trace (the last one is summarised)")
a = ap.parse_args()

rows = []
with open(a.trace) as f:
    for r in csv.DictReader(f):
        rows.append((r["Kernel_Name"], int(r["Thread_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
rows.sort(key=lambda t: t[2])


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("mcx::", "")


threads = sorted({t for _, t, _, _ in rows})
# the CG kernels of the last solve: the launches after the last k_cg_init of each thread
per_thread = collections.defaultdict(list)
for n, t, s, e in rows:
    per_thread[t].append((short(n), s, e))
summary = {}
for t in threads:
    ks = per_thread[t]
    inits = [q for q, (n, _, _) in enumerate(ks) if n.startswith("k_cg_init")]
    if not inits:
        continue
    last = ks[inits[-1]:]
    agg = collections.defaultdict(lambda: [0, 0])
    for n, s, e in last:
        agg[n][0] += 1
        agg[n][1] += e - s
    summary[t] = {n: {"calls": c, "total_us": tot / 1e3, "avg_us": tot / c / 1e3,
                      "per_iter_us": tot / 1e3 / a.its if a.its else None} for n, (c, tot) in agg.items()}
    # span of the last solve on this thread and the union of all threads' busy time in it
    summary[t]["_span_us"] = (last[-1][2] - last[0][1]) / 1e3
names = sorted({n for t in summary for n in summary[t] if not n.startswith("_")})
print(f"threads (ranks): {len(summary)}")
print(f"{'kernel':60s} " + " ".join(f"{'r' + str(q):>10s}" for q in range(len(summary))) + "   (us per CG iteration)")
for n in names:
    vals = []
    for t in summary:
        v = summary[t].get(n)
        vals.append(f"{(v['per_iter_us'] if a.its else v['avg_us']):10.2f}" if v else f"{'-':>10s}")
    print(f"{n[:60]:60s} " + " ".join(vals))
print(json.dumps(summary))
