#!/bin/bash
# GPU box: one rocprofv3 --pmc pass per ragged-gap case of
# scripts/dev/case_run.py with the given counters (mind the per-block pass
# limits: 4 TCC, 4 TCP, 8 SQ ...), then each counter's mean per dispatch
# (the first launch skipped).
# usage: scripts/dev/pmc_cases.sh OUTDIR "COUNTER ..." [cases ...]
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pmc}; shift
CTRS=$1; shift
CASES=${@:-F16 FB16 F4M P28 C28 R28}
mkdir -p $O
for c in $CASES; do
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $O/$c -o p -- \
    python3 scripts/dev/case_run.py $c 4 > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
done
python3 - "$O" $CASES <<'EOF'
import csv, glob, sys, collections
o = sys.argv[1]
for c in sys.argv[2:]:
    f = glob.glob(f"{o}/{c}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "obfs_kernel" in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(per)[1:] or sorted(per)
    avg = {k: sum(per[i][k] for i in ids) / len(ids) for k in sorted(per[ids[0]])}
    print(f"{c:5s} " + " ".join(f"{k} {v:.5g}" for k, v in avg.items()), flush=True)
EOF
