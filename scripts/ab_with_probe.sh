#!/bin/bash
# On the GPU box: kernel variants (build/var) and the copy probe's matching
# pattern in ONE call, so box-to-box bandwidth differences cancel.
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; mkdir -p $O
timeout -k 10 300 python scripts/probe_copy.py occ > $O/probe_occ.log 2>&1 || exit 1
REPS=${REPS:-3} timeout -k 10 600 bash scripts/run_variants.sh ${1:-ab}
