#!/bin/bash
# GPU box: parity of every build/var/lib_*.so on the core parity file (one
# process per lib).
cd $GRAFT_REPO_ROOT
N=${1:-r2pt}; T=${2:-tests/test_gpu_parity.py}
mkdir -p gpurun_out/$N
for L in build/var/lib_*.so; do
  n=$(basename $L .so)
  SQOBFS_LIB=$L timeout -k 10 300 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$N/pytest_$n.log 2>&1 || { echo "$n PARITY FAILED"; tail -30 gpurun_out/$N/pytest_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/$N/pytest_$n.log)"
done
