#!/bin/bash
# GPU box: kernel variants (build/var) + copy-probe occupancy calibration
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r2var}
REPS=3 timeout -k 10 500 bash scripts/run_variants.sh ${1:-r2var} > gpurun_out/${1:-r2var}.txt 2>&1 && \
timeout -k 10 200 python scripts/probe_copy.py occ > gpurun_out/${1:-r2var}_probe.txt 2>&1
