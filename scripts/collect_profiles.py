"""Copy a scripts/final_profiles.sh run (gpurun_out/<tag>/) into the tracked
profiles/ tree: per-config kernel stats, PMC counter summaries and bench
lines under profiles/r01/, the per-config HBM-traffic files bench.py reads
under profiles/, and the QUIC kernel trace.
usage: python scripts/collect_profiles.py [tag]"""
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "final"
src = os.path.join(REPO, "gpurun_out", tag)
dst = os.path.join(REPO, "profiles", "r01")
for c in sorted(os.listdir(src)):
    d = os.path.join(src, c)
    if not os.path.exists(os.path.join(d, "summary.json")):
        continue
    shutil.copy(os.path.join(d, "kernel_stats.csv"), f"{dst}/kernel_stats_{c}.csv")
    shutil.copy(os.path.join(d, "bench_kt.json"), f"{dst}/bench_kt_{c}.json")
    s = json.load(open(os.path.join(d, "summary.json")))
    json.dump(s, open(f"{dst}/pmc_{c}_counters.json", "w"), indent=1)
    top = os.path.join(REPO, "profiles", f"pmc_{c}.json")
    t = json.load(open(top)) if os.path.exists(top) else {}
    t.update(hbm_bytes_per_launch=s["hbm_bytes_per_launch"],
             hbm_read_bytes=s["hbm_read_bytes_corrected"], hbm_write_bytes=s["hbm_write_bytes"])
    json.dump(t, open(top, "w"), indent=1)
    print(c, s["hbm_bytes_per_launch"])
b = os.path.join(src, "bench_default.json")
if os.path.exists(b):
    shutil.copy(b, f"{dst}/bench_salamander-1m.json")
q = os.path.join(src, "quic")
if os.path.isdir(q):
    os.makedirs(f"{dst}/quic", exist_ok=True)
    for sub, name in (("kt", "aes_128_gcm"), ("kt2", "chacha20_poly1305")):
        f = os.path.join(q, sub, "kt_kernel_stats.csv")
        if os.path.exists(f):
            shutil.copy(f, f"{dst}/quic/kernel_stats_{name}.csv")
    shutil.copy(os.path.join(q, "bench_quic.json"), f"{dst}/quic/bench_quic.json")
