#!/bin/bash
# GPU box: a subset (or all) of the GPU tests, then timing variants in build/var
cd $GRAFT_REPO_ROOT
N=${1:-r2tv}; T=${2:-tests}
mkdir -p gpurun_out/$N
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$N/pytest.log 2>&1 || { tail -40 gpurun_out/$N/pytest.log; exit 1; }
tail -2 gpurun_out/$N/pytest.log
if ls build/var/lib_*.so >/dev/null 2>&1; then
  REPS=${REPS:-3} timeout -k 10 700 bash scripts/run_variants.sh $N/var > gpurun_out/$N/var.txt 2>&1
  rc=$?; cat gpurun_out/$N/var.txt; exit $rc
fi
