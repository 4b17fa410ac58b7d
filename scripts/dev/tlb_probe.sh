#!/bin/bash
# GPU box: address-translation counters (TCP UTCL1) per dispatch for the
# ragged-gap cases of scripts/dev/case_run.py, one rocprofv3 --pmc pass per
# case (4 TCP counters: the pass limit), then a summary per case.
# usage: scripts/dev/tlb_probe.sh OUTDIR [cases ...]
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-tlb}; shift
CASES=${@:-F16 FB16 F4M P28 C28 R28}
mkdir -p $O
for c in $CASES; do
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
    TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum --output-format csv -d $O/$c -o p -- \
    python3 scripts/dev/case_run.py $c 4 > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
  echo "$c done"
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
    ids = sorted(per)[1:] or sorted(per)  # (past the first launch)
    avg = {k: sum(per[i][k] for i in ids) / len(ids) for k in per[ids[0]]}
    miss, hit, req = (avg.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0),
                      avg.get("TCP_UTCL1_TRANSLATION_HIT_sum", 0), avg.get("TCP_UTCL1_REQUEST_sum", 0))
    print(f"{c:5s} dispatches {len(ids)} request {req:.4g} hit {hit:.4g} miss {miss:.4g} "
          f"miss/req {miss / max(req, 1):.4%} multi-miss stall "
          f"{avg.get('TCP_UTCL1_STALL_MULTI_MISS_sum', 0):.4g}")
EOF
