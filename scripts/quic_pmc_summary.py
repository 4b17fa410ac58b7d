"""Per-kernel averages of the QUIC PMC passes (scripts/quic_pmc.sh) and
the VALU roofline of each QUIC kernel: VALU wave-instructions per launch
over the kernel's average duration (kernel trace), against the MI355X VALU
issue rate: 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction.
Writes <dir>/quic_summary.json."""
import csv
import glob
import json
import os
import sys

PEAK = 256 * 4 * 2.4e9 / 2  # wave-instructions / s
d = sys.argv[1]
cnt = {}
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "quic" not in k:
            continue
        cnt.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
dur = {}
for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "quic" in k:
            dur.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = {"peak_valu_wave_instr_per_s": PEAK, "kernels": {}}
for k, c in cnt.items():
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    e = {"counters": avg}
    if k in dur and "SQ_INSTS_VALU" in avg:
        us = sum(dur[k]) / len(dur[k])
        e["kernel_avg_us"] = round(us, 2)
        e["valu_instr_per_s"] = avg["SQ_INSTS_VALU"] / (us * 1e-6)
        e["valu_frac_of_peak"] = round(e["valu_instr_per_s"] / PEAK, 4)
    out["kernels"][k] = e
json.dump(out, open(os.path.join(d, "quic_summary.json"), "w"), indent=1)
for k, e in out["kernels"].items():
    print(k[:90], e.get("kernel_avg_us"), e.get("valu_frac_of_peak"),
          round(e["counters"].get("SQ_INSTS_VALU", 0) / 1048576, 1), "VALU/pkt")
