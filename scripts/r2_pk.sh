#!/bin/bash
# GPU box: parity tests of the current build, then the timing variants in build/var
set -o pipefail
cd $GRAFT_REPO_ROOT
N=${1:-r2pk}
mkdir -p gpurun_out/$N
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$N/pytest.log 2>&1 || { tail -30 gpurun_out/$N/pytest.log; exit 1; }
tail -2 gpurun_out/$N/pytest.log
REPS=3 timeout -k 10 600 bash scripts/run_variants.sh $N/var > gpurun_out/$N/var.txt 2>&1
cat gpurun_out/$N/var.txt
