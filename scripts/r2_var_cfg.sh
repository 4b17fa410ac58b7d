#!/bin/bash
# GPU box: timing variants in build/var on several bench configs
cd $GRAFT_REPO_ROOT
N=$1; shift
mkdir -p gpurun_out/$N
for cfg in "$@"; do
  REPS=${REPS:-2} timeout -k 10 600 bash scripts/run_variants.sh $N/$cfg --config $cfg > gpurun_out/$N/$cfg.txt 2>&1 || { cat gpurun_out/$N/$cfg.txt; exit 1; }
  echo "== $cfg"; cat gpurun_out/$N/$cfg.txt
done
