#!/bin/bash
# GPU box: the AES-128-GCM kernels (scripts/quic_prof.py: seal + open of 1M x
# 1,361-B packets, one key) under a kernel trace and two PMC passes, then a
# summary per kernel: average duration, VALU / LDS wave-instructions per
# packet, the share of wave time spent waiting, and the effective clock.
# usage: scripts/dev/gcm_pmc.sh OUTDIR [suite=1]
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
SUITE=${2:-1}
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
  python3 scripts/quic_prof.py $SUITE 6 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
           "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p -- \
    python3 scripts/quic_prof.py $SUITE 2 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - "$O" <<'EOF' | tee $O/summary.txt
import csv, glob, statistics, sys, collections
o = sys.argv[1]
N = 1 << 20
st = glob.glob(f"{o}/kt/**/*kernel_stats.csv", recursive=True)[0]
dur = {r["Name"]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(st)) if "quic" in r["Name"]}
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{o}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "quic" not in r["Kernel_Name"]:
            continue
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        per[r["Kernel_Name"]][r["Counter_Name"]].append((float(r["Counter_Value"]), us))
for k, d in per.items():
    med = {c: statistics.median(v for v, _ in x) for c, x in d.items()}
    us = statistics.median(u for _, u in d.get("GRBM_GUI_ACTIVE", [(0, 1)]))
    line = f"{k[:60]:60s} avg {dur.get(k, 0):8.1f} us"
    if "SQ_INSTS_VALU" in med:
        line += f" valu/pkt {med['SQ_INSTS_VALU'] / N:7.1f} lds/pkt {med['SQ_INSTS_LDS'] / N:6.1f}"
        line += f" wait {med['SQ_WAIT_ANY'] / max(med['SQ_WAVE_CYCLES'], 1):.3f}"
        line += f" valu_active {med.get('SQ_ACTIVE_INST_VALU', 0) / max(med['SQ_WAVE_CYCLES'], 1):.3f}"
    if "GRBM_GUI_ACTIVE" in med:
        line += f" clock {med['GRBM_GUI_ACTIVE'] / 8 / us:.0f} MHz"
        line += f" ldsconf {med['SQ_LDS_BANK_CONFLICT'] / max(med['SQ_LDS_IDX_ACTIVE'], 1):.3f}"
    print(line)
EOF
