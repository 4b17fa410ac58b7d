#!/bin/bash
# GPU box: kernel trace (+stats) and PMC passes of bench.py for one config.
# usage: scripts/profile.sh OUTDIR [bench args]   (each pass its own run)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e "$@" > $O/kt.json 2> $O/kt.log \
  || { echo "kernel trace failed"; tail -5 $O/kt.log; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p -- \
    python bench.py --steps 5 --warmup 1 --warmup-s 0 --no-cpu-baseline --no-e2e "$@" > $O/p$i.log 2>&1 \
    || { echo "pass $i ($grp) failed"; tail -5 $O/p$i.log; exit 1; }
done
python scripts/pmc_summary.py $O
# keep the outputs small (gpurun returns at most 64 MiB): the obfs_kernel rows
# of every CSV, nothing else
python - "$O" <<'PY'
import csv, glob, os, sys
for f in glob.glob(os.path.join(sys.argv[1], "**", "*.csv"), recursive=True):
    rows = list(csv.reader(open(f)))
    if not rows or "Kernel_Name" not in rows[0]:
        continue
    k = rows[0].index("Kernel_Name")
    keep = [rows[0]] + [r for r in rows[1:] if len(r) > k and "obfs_kernel" in r[k]]
    csv.writer(open(f, "w", newline="")).writerows(keep)
PY
du -sh $O
