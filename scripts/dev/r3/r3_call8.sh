#!/bin/bash
# GPU box: workgroup size (waves per block) variants: parity, then timing in
# interleaved processes (unit_sweep per lib, two rounds).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c8; mkdir -p $O
SQOBFS_LIB=build/var/lib_b64.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_b64.log 2>&1 || { tail -30 $O/pt_b64.log; exit 1; }
echo "b64 $(tail -1 $O/pt_b64.log)"
for r in 1 2; do
  for L in b256 b64 b128; do
    for c in salamander-1m salamander-ragged-4m; do
      w="16 14"; [ $c = salamander-ragged-4m ] && w="28 24"
      SQOBFS_LIB=build/var/lib_$L.so timeout -k 10 300 python -u scripts/dev/unit_sweep.py $c "$w" 3 > $O/${L}_${c}_r$r.txt 2>&1 || { tail -5 $O/${L}_${c}_r$r.txt; exit 1; }
      grep ppw $O/${L}_${c}_r$r.txt | sed "s/^/$L r$r /" | cut -c1-90
    done
  done
done
