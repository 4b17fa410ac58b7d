"""Average each PMC counter over the obfs_kernel dispatches of a pmc.sh run.
Writes <dir>/summary.json.  Byte conversions per MI355X_MICROARCH.md:
FETCH_SIZE/WRITE_SIZE are KiB; FETCH_SIZE reads half the bytes of a wide
coalesced stream on gfx950, so HBM read bytes = 2 * FETCH_SIZE * 1024."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
vals = {}
dur = []
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "obfs_kernel" not in r["Kernel_Name"] and "probe" not in r["Kernel_Name"]:
            continue
        vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
out = {k: sum(v) / len(v) for k, v in vals.items()}
if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
    out["hbm_read_bytes_corrected"] = 2 * out["FETCH_SIZE"] * 1024
    out["hbm_write_bytes"] = out["WRITE_SIZE"] * 1024
    out["hbm_bytes_per_launch"] = out["hbm_read_bytes_corrected"] + out["hbm_write_bytes"]
json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
