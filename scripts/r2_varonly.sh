#!/bin/bash
# GPU box: timing variants in build/var only (REPS interleaved passes)
cd $GRAFT_REPO_ROOT
N=${1:-r2v}; shift
mkdir -p gpurun_out/$N
REPS=${REPS:-3} timeout -k 10 900 bash scripts/run_variants.sh $N/var "$@" > gpurun_out/$N/var.txt 2>&1
rc=$?; cat gpurun_out/$N/var.txt; exit $rc
