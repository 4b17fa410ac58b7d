#!/bin/bash
# GPU box: profiles of every config (kernel trace + PMC passes), then the
# driver's bench command and every config / direction with the shipped lib.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r3f}
timeout -k 10 1000 bash scripts/r2_profile_all.sh $T > gpurun_out/$T.log 2>&1 || { tail -20 gpurun_out/$T.log; exit 1; }
tail -3 gpurun_out/$T.log
timeout -k 10 800 bash scripts/r2_configs.sh $T/cfg > gpurun_out/$T/cfg.txt 2>&1 || { tail -20 gpurun_out/$T/cfg.txt; exit 1; }
cat gpurun_out/$T/cfg.txt
