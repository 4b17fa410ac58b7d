#!/bin/bash
# GPU box: parity of every build/var/lib_*.so (tests/test_gpu_parity.py, one
# process per lib), then interleaved timing on each config given.
cd $GRAFT_REPO_ROOT
N=${1:-r2pc}; shift
mkdir -p gpurun_out/$N
for L in build/var/lib_*.so; do
  n=$(basename $L .so)
  SQOBFS_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$N/pytest_$n.log 2>&1 || { echo "$n PARITY FAILED"; tail -30 gpurun_out/$N/pytest_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/$N/pytest_$n.log)"
done
for c in "$@"; do
  echo "== $c"
  REPS=${REPS:-3} timeout -k 10 900 bash scripts/run_variants.sh $N/var_$c --config $c > gpurun_out/$N/var_$c.txt 2>&1 || { cat gpurun_out/$N/var_$c.txt; exit 1; }
  cat gpurun_out/$N/var_$c.txt
done
