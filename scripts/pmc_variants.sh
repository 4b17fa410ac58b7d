#!/bin/bash
# On the GPU box: HBM bytes per launch (FETCH_SIZE and WRITE_SIZE in separate
# passes, scripts/pmc_summary.py corrections) of configs[1] for every
# build/var/lib_*.so.
export TMPDIR=/tmp
O=gpurun_out/${1:-pmcvar}; mkdir -p $O
for L in build/var/lib_*.so; do
  n=$(basename $L .so); mkdir -p $O/$n
  SQOBFS_LIB=$L timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$n/p1 -o p -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/$n/p1.log 2>&1 || { echo "$n p1 failed"; exit 1; }
  SQOBFS_LIB=$L timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$n/p2 -o p -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/$n/p2.log 2>&1 || { echo "$n p2 failed"; exit 1; }
  python scripts/pmc_summary.py $O/$n > /dev/null || exit 1
  python -c "import json; d=json.load(open('$O/$n/summary.json')); print('$n', 'read', round(d['hbm_read_bytes_corrected']/1e9,4), 'write', round(d['hbm_write_bytes']/1e9,4), 'GB')"
done
