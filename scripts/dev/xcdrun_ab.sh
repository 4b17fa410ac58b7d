#!/bin/bash
# GPU box: parity of the XCD-runs variants (build/ab/lib_run*.so), then the
# ragged probe's cases and the size ladder with base vs runs, in one process.
# usage: scripts/dev/xcdrun_ab.sh OUTDIR "variant ..."
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-xrun}; V=$2
mkdir -p $O
L="build/ab/lib_base.so"
for v in $V; do
  SQOBFS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_fuzz.py tests/test_gpu_scatter.py tests/test_gpu_fullsize.py -m gpu -x -q \
    --timeout 180 --timeout-method thread -k "not bench" > $O/parity_$v.log 2>&1 \
    || { echo "parity $v failed"; tail -30 $O/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $O/parity_$v.log)"
  L="$L build/ab/lib_$v.so"
done
for d in obfuscate deobfuscate; do
  timeout -k 10 500 python -u scripts/dev/ragged_split.py $d 5 $L > $O/split_$d.txt 2>&1 \
    || { echo "split $d failed"; tail -5 $O/split_$d.txt; exit 1; }
  SPLIT_CASES=ladder timeout -k 10 500 python -u scripts/dev/ragged_split.py $d 5 $L \
    > $O/ladder_$d.txt 2>&1 || { echo "ladder $d failed"; tail -5 $O/ladder_$d.txt; exit 1; }
done
grep -h median $O/split_*.txt $O/ladder_*.txt
