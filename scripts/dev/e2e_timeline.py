"""Dev (container): one sqobfs_run_host call's timeline from a rocprofv3
--hip-trace --memory-copy-trace --kernel-trace run of scripts/dev/e2e_trace.py
(times in us from the call's first HIP API call): each API call, and the copy
or kernel it started.  usage: e2e_timeline.py TRACE_DIR [call index]"""
import csv
import os
import sys

d = sys.argv[1]
ci = int(sys.argv[2]) if len(sys.argv) > 2 else 5
keep = ("hipMemcpyAsync", "hipMemcpy2DAsync", "hipStreamSynchronize", "hipLaunchKernel",
        "hipPointerGetAttributes", "hipEventSynchronize")
api = [r for r in csv.DictReader(open(os.path.join(d, "tr_hip_api_trace.csv")))
       if r["Function"] in keep]
cp = {int(r["Correlation_Id"]): r for r in csv.DictReader(open(os.path.join(d, "tr_memory_copy_trace.csv")))}
ks = {int(r["Correlation_Id"]): r for r in csv.DictReader(open(os.path.join(d, "tr_kernel_trace.csv")))}
calls, cur = [], []
for r in sorted(api, key=lambda r: int(r["Start_Timestamp"])):
    cur.append(r)
    if r["Function"] == "hipStreamSynchronize":
        calls.append(cur)
        cur = []
c = calls[ci]
t0 = int(c[0]["Start_Timestamp"])


def us(x):
    return (int(x) - t0) / 1e3


for r in c:
    cid = int(r["Correlation_Id"])
    extra = ""
    if cid in cp:
        x = cp[cid]
        extra = f"  copy {x['Direction'][12:]:15s} {us(x['Start_Timestamp']):8.1f} - {us(x['End_Timestamp']):8.1f}"
    if cid in ks:
        x = ks[cid]
        extra = f"  kernel {us(x['Start_Timestamp']):8.1f} - {us(x['End_Timestamp']):8.1f} {x['Kernel_Name'][:34]}"
    print(f"{r['Function'][:22]:22s} {us(r['Start_Timestamp']):8.1f} {us(r['End_Timestamp']):8.1f}{extra}")
