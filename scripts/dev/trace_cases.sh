#!/bin/bash
# GPU box: the kernel time of each ragged-gap case of scripts/dev/case_run.py
# in a process of its own (rocprofv3 --kernel-trace; LAUNCHES launches, the
# last 20 timed: a fresh process's first ~30 run up to 10 % slow), against ragged_split.py, which holds every case's
# buffers in one process.
# usage: scripts/dev/trace_cases.sh OUTDIR [LAUNCHES [cases ...]]
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-tc}; shift
N=${1:-12}; shift
CASES=${@:-F16 FB16 F4M P28 C28 R28}
mkdir -p $O
for c in $CASES; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/$c -o kt -- \
    python3 scripts/dev/case_run.py $c $N > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
done
python3 - "$O" $CASES <<'EOF'
import csv, glob, statistics, sys
o = sys.argv[1]
B = {"F16": (1 << 20) * 2716, "F4M": (1 << 22) * 2716, "FB16": 2372000 * 2716,
     "P28": (1 << 20) * 1532, "C28": (1 << 22) * 1532, "R28": (1 << 22) * 1532}  # (R28: mean)
for c in sys.argv[2:]:
    f = glob.glob(f"{o}/{c}/**/*kernel_trace.csv", recursive=True)[0]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
         for r in csv.DictReader(open(f)) if "obfs_kernel" in r["Kernel_Name"]][-20:]
    med = statistics.median(d)
    b = B[c]
    print(f"{c:5s} launches {len(d)} median {med:8.1f} us" +
          (f"  frac {b / med / 8e6:.4f}" if b else ""), flush=True)
EOF
