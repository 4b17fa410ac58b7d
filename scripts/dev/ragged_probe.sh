#!/bin/bash
# GPU box: the ragged-gap experiments ("Ragged batches").
#   1. ragged_split.py: configs[3] beside same-mean constant lengths, 16
#      packets per wave and byte-balanced units, for every lib given
#   2. timeline.py (a -DSQ_TIMELINE=1 build, build/ab/lib_tl.so) of configs[3]
#      and configs[1]: phase medians and mean resident waves
# usage: scripts/dev/ragged_probe.sh OUTDIR ROUNDS lib.so ...
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ragged}; shift
R=${1:-5}; shift
mkdir -p $O
for d in obfuscate deobfuscate; do
  timeout -k 10 400 python -u scripts/dev/ragged_split.py $d $R "$@" > $O/split_$d.txt 2>&1 \
    || { tail -5 $O/split_$d.txt; exit 1; }
done
if [ -f build/ab/lib_tl.so ]; then
  for c in salamander-ragged-4m salamander-1m; do
    for d in obfuscate deobfuscate; do
      SQOBFS_LIB=build/ab/lib_tl.so timeout -k 10 200 python -u scripts/dev/timeline.py $c 0 $d \
        > $O/timeline_${c}_$d.json 2> $O/tl_err.txt || { tail -5 $O/tl_err.txt; exit 1; }
    done
  done
fi
grep -h "median" $O/split_*.txt
