#!/bin/bash
# On the GPU box: bench one lib over the three layouts.
export TMPDIR=/tmp
O=gpurun_out/${1:-lay}; shift; mkdir -p $O
for L in ${LIBS:-default}; do
  for lay in dense slot16 inplace; do
    lib=""; [ "$L" != default ] && lib=$L
    SQOBFS_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --layout $lay "$@" > $O/$(basename $L .so)_$lay.json 2> $O/err_$lay.txt || { echo "FAILED $L $lay"; tail -3 $O/err_$lay.txt; exit 1; }
    python -c "import json;d=json.load(open('$O/$(basename $L .so)_$lay.json'));r=d['roofline'];print('$(basename $L .so)', '$lay', r['kernel_avg_us'], r['frac'], d['parity_spot_check'])"
  done
done
