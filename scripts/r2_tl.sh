#!/bin/bash
# GPU box: timing variants in build/var (REPS interleaved passes), then the
# per-wave timeline of every build/tl/lib_*.so (scripts/dev/timeline.py).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
N=${1:-r2tl}; shift
mkdir -p gpurun_out/$N
if ls build/var/lib_*.so >/dev/null 2>&1; then
  REPS=${REPS:-3} timeout -k 10 900 bash scripts/run_variants.sh $N/var "$@" > gpurun_out/$N/var.txt 2>&1 || { cat gpurun_out/$N/var.txt; exit 1; }
  cat gpurun_out/$N/var.txt
fi
for L in build/tl/lib_*.so; do
  [ -e "$L" ] || continue
  n=$(basename $L .so)
  SQOBFS_LIB=$L timeout -k 10 120 python scripts/dev/timeline.py ${TLCFG:-salamander-1m} > gpurun_out/$N/$n.json 2> gpurun_out/$N/$n.err || { echo "$n FAILED"; tail -5 gpurun_out/$N/$n.err; exit 1; }
done
