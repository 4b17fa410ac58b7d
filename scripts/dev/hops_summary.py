"""Summarise a `lat_bench hops` JSON (profiles/r05/engine/hops_*.json): per
offered rate and mode, the medians (and ranges) of host CPU seconds per GiB,
payload GiB/s, launches and batches per launch over the repetitions.
usage: hops_summary.py FILE"""
import json
import statistics as S
import sys
from collections import defaultdict

runs = json.load(open(sys.argv[1]))["hops"]
g = defaultdict(list)
for r in runs:
    g[(r["offered_gib_s"], r["mode"])].append(r)
print("| offered | mode | CPU s/GiB median (range) | GiB/s | launches | batches/launch | CPU-path batches |")
print("|---|---|---|---|---|---|---|")
for (rate, mode), rs in sorted(g.items(), key=lambda x: (x[0][0] or 1e9, x[0][1])):
    c = [r["cpu_s_per_gib"] for r in rs]
    print(f"| {rate or 'unpaced'} | {mode} | {S.median(c):.2f} ({min(c):.2f}-{max(c):.2f}) | "
          f"{S.median(r['payload_gib_s'] for r in rs):.2f} | "
          f"{S.median(r['launches'] for r in rs):.0f} | "
          f"{S.median(r['batches_per_launch'] for r in rs):.2f} | "
          f"{S.median(r['cpu_batches'] for r in rs):.0f} of {S.median(r['batches'] for r in rs):.0f} |")
