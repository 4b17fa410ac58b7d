#!/bin/bash
# GPU box: VERDICT r5 item 2's control.  For each ragged-gap case, in
# processes of their own: the obfuscation kernel (scripts/dev/case_run.py)
# and a plain dense dwordx4 nontemporal copy of the same footprint
# (scripts/dev/copy_footprint.py, both patterns), each under
# rocprofv3 --kernel-trace (the last launches' median), then one
# --pmc GRBM_GUI_ACTIVE pass each for the effective shader clock
# (GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time, MI355X_MICROARCH.md).
# usage: scripts/dev/footprint.sh OUTDIR [LAUNCHES [cases ...]]
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-fp}; shift
N=${1:-16}; shift
CASES=${@:-F16 FB16 F4M P28 C28 R28}
mkdir -p $O
test -f build/libsqprobe.so || { echo "build/libsqprobe.so missing"; exit 1; }
for c in $CASES; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/k_$c -o kt -- \
    python3 scripts/dev/case_run.py $c $N > $O/k_$c.log 2>&1 || { tail -5 $O/k_$c.log; exit 1; }
  for p in 1 0; do
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/c${p}_$c -o kt -- \
      python3 scripts/dev/copy_footprint.py $c $N $p > $O/c${p}_$c.log 2>&1 || { tail -5 $O/c${p}_$c.log; exit 1; }
  done
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d $O/kp_$c -o p -- \
    python3 scripts/dev/case_run.py $c 6 > $O/kp_$c.log 2>&1 || { tail -5 $O/kp_$c.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d $O/cp_$c -o p -- \
    python3 scripts/dev/copy_footprint.py $c 6 1 > $O/cp_$c.log 2>&1 || { tail -5 $O/cp_$c.log; exit 1; }
  echo "$c done"
done
python3 - "$O" $CASES <<'EOF' | tee $O/summary.txt
import csv, glob, statistics, sys
o = sys.argv[1]
# algorithmic bytes per launch (payload in + salt + payload out); R28: mean
B = {"F16": (1 << 20) * 2716, "F4M": (1 << 22) * 2716, "FB16": 2372000 * 2716,
     "P28": (1 << 20) * 1532, "C28": (1 << 22) * 1532, "R28": (1 << 22) * 1532,
     "F16M": (1 << 24) * 2716}
CB = {"F16": (1 << 20) * 1358, "F4M": (1 << 22) * 1358, "FB16": 2372000 * 1358,
      "P28": (1 << 20) * 766, "C28": (1 << 22) * 766, "R28": (1 << 22) * 766,
      "F16M": (1 << 24) * 1358}
def med(d, key):
    f = glob.glob(f"{o}/{d}/**/*kernel_trace.csv", recursive=True)[0]
    x = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
         for r in csv.DictReader(open(f)) if key in r["Kernel_Name"]]
    x = x[len(x) // 2:]
    return statistics.median(x), len(x)
def clock(d, key):
    f = glob.glob(f"{o}/{d}/**/*counter_collection.csv", recursive=True)[0]
    x = [float(r["Counter_Value"]) / 8 / ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
         for r in csv.DictReader(open(f)) if key in r["Kernel_Name"] and r["Counter_Name"].startswith("GRBM_GUI_ACTIVE")]
    x = x[1:] or x
    return statistics.median(x)
print("case  kernel_us frac  | copy(pat1)_us frac | copy(pat0)_us frac | kernel/best-copy | clock MHz kernel / copy")
for c in sys.argv[2:]:
    k, nk = med(f"k_{c}", "obfs_kernel")
    c1, _ = med(f"c1_{c}", "probe")
    c0, _ = med(f"c0_{c}", "probe")
    cb = (CB[c] + 21759) // 21760 * 21760 * 2
    fk, f1, f0 = B[c] / k / 8e6, cb / c1 / 8e6, cb / c0 / 8e6
    print(f"{c:5s} {k:8.1f} {fk:.4f} | {c1:8.1f} {f1:.4f} | {c0:8.1f} {f0:.4f} | "
          f"{fk / max(f1, f0):.4f} | {clock(f'kp_{c}', 'obfs_kernel'):.0f} / {clock(f'cp_{c}', 'probe'):.0f}",
          flush=True)
EOF
