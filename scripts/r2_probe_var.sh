#!/bin/bash
# GPU box: a copy-probe mode, then the timing variants in build/var
cd $GRAFT_REPO_ROOT
N=${1:-r2pv}; M=${2:-groups}
mkdir -p gpurun_out/$N
timeout -k 10 200 python scripts/probe_copy.py $M > gpurun_out/$N/probe.txt 2>&1 || exit 1
grep TBps gpurun_out/$N/probe.txt
REPS=${REPS:-3} timeout -k 10 700 bash scripts/run_variants.sh $N/var > gpurun_out/$N/var.txt 2>&1
rc=$?; cat gpurun_out/$N/var.txt; exit $rc
