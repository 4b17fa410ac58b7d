"""Copy a scripts/profile_configs.sh run (gpurun_out/<tag>/) into profiles/<round>/:
per config the kernel-trace stats, the PMC summary and the HBM-traffic file
bench.py reads (profiles/<round>/pmc_<config>.json).
usage: python scripts/collect_profiles.py TAG [ROUND (default r03)]"""
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(REPO, "gpurun_out", sys.argv[1])
rnd = sys.argv[2] if len(sys.argv) > 2 else "r03"
dst = os.path.join(REPO, "profiles", rnd)
os.makedirs(dst, exist_ok=True)
for d in sorted(glob.glob(os.path.join(src, "*"))):
    if not os.path.isdir(d):
        continue
    cfg = os.path.basename(d)
    st = glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True)
    if st:
        shutil.copy(st[0], os.path.join(dst, f"kernel_stats_{cfg}.csv"))
    tr = glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True)
    if tr:
        # the timed launches are the `steps` obfs_kernel dispatches before the
        # bench's per-launch pass (min(steps, 20) more, when its line has
        # kernel_each_rule), or the last `steps` (earlier bench lines); the
        # kernel-stats average also holds the cold first launches of warm-up
        import csv
        rows = [r for r in csv.DictReader(open(tr[0])) if "obfs_kernel" in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        kt = json.loads(open(os.path.join(d, "kt.json")).read().strip().splitlines()[-1])
        k = kt["steps"]
        each = min(k, 20) if "kernel_each_rule" in kt["roofline"] else 0
        last = rows[len(rows) - each - k:len(rows) - each]
        us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in last]
        span = (int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])) / 1e3 / k
        json.dump({"kernel": last[-1]["Kernel_Name"], "dispatches": len(rows),
                   "timed_dispatches": len(us), "timed_avg_us": round(sum(us) / len(us), 2),
                   "timed_min_us": round(min(us), 2), "timed_max_us": round(max(us), 2),
                   "timed_span_per_dispatch_us": round(span, 2),
                   "bench_kernel_avg_us_same_run": kt["roofline"]["kernel_avg_us"],
                   "lds_bytes": last[-1]["LDS_Block_Size"],
                   "grid": last[-1]["Grid_Size_X"], "workgroup": last[-1]["Workgroup_Size_X"],
                   "source": "rocprofv3 --kernel-trace --stats (scripts/profile.sh)"},
                  open(os.path.join(dst, f"kernel_trace_timed_{cfg}.json"), "w"), indent=1)
    summ = os.path.join(d, "summary.json")
    if not os.path.exists(summ):
        continue
    s = json.load(open(summ))
    shutil.copy(summ, os.path.join(dst, f"pmc_{cfg}_counters.json"))
    kt = json.loads(open(os.path.join(d, "kt.json")).read().strip().splitlines()[-1])
    alg = kt["roofline"]["algorithmic_bytes_per_launch"]
    out = {"hbm_bytes_per_launch": s["hbm_bytes_per_launch"],
           "hbm_read_bytes": s["hbm_read_bytes_corrected"],
           "hbm_write_bytes": s["hbm_write_bytes"],
           "algorithmic_bytes_per_launch": alg,
           "traffic_over_algorithmic": round(s["hbm_bytes_per_launch"] / alg, 4),
           "source": f"profiles/{rnd}/pmc_{cfg}_counters.json: rocprofv3 --pmc FETCH_SIZE and "
                     "--pmc WRITE_SIZE in separate passes (scripts/profile.sh), bench.py "
                     "--steps 5; read = 2*FETCH_SIZE*1024 (gfx950 half-count correction), "
                     "write = WRITE_SIZE*1024",
           "kernel": kt["roofline"].get("kernel")}
    json.dump(out, open(os.path.join(dst, f"pmc_{cfg}.json"), "w"), indent=1)
    print(cfg, out["traffic_over_algorithmic"], kt["roofline"]["kernel_avg_us"], kt["roofline"]["frac"])
b = os.path.join(src, "bench_default.json")
if os.path.exists(b):
    shutil.copy(b, os.path.join(dst, "bench_salamander-1m.json"))
