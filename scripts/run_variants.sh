#!/bin/bash
# On the GPU box: bench every build/var/lib_*.so (kernel avg us, parity).
export TMPDIR=/tmp
O=gpurun_out/${1:-var}; shift; mkdir -p $O
for L in build/var/lib_*.so; do
  n=$(basename $L .so)
  SQOBFS_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "$n FAILED"; tail -3 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));r=d['roofline'];print('$n', r['kernel_avg_us'], r['frac'], d['parity_spot_check'])"
done
