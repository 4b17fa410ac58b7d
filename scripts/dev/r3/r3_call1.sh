#!/bin/bash
# GPU box: unit-size parity test, the two-lane-hash variant's parity, the
# in-process unit-size sweep per config, then base vs two-lane hash timing.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c1; mkdir -p $O
PT="python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_parity.py -k unit_sizes > $O/us_test.log 2>&1 || { tail -30 $O/us_test.log; exit 1; }
tail -1 $O/us_test.log
SQOBFS_LIB=build/var/lib_h2.so timeout -k 10 300 $PT tests/test_gpu_parity.py > $O/h2_test.log 2>&1 || { tail -30 $O/h2_test.log; exit 1; }
tail -1 $O/h2_test.log
for c in salamander-1m xplus-1m salamander-ragged-4m; do
  timeout -k 10 200 python -u scripts/dev/unit_sweep.py $c "16 20 24 26 28 30 31 32 34 36 40 48 56" 7 > $O/us_$c.txt 2>&1 || { tail -5 $O/us_$c.txt; exit 1; }
  grep ppw $O/us_$c.txt
done
REPS=5 timeout -k 10 400 bash scripts/run_variants.sh r3c1/var --unit-packets 31 > $O/var.txt 2>&1 || { cat $O/var.txt; exit 1; }
cat $O/var.txt
