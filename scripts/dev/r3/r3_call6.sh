#!/bin/bash
# GPU box: stream step (U) and late-keystream variants at the byte-sized
# units, in-process A/B (dev builds in build/var).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c6; mkdir -p $O
for u in 2 8; do
  SQOBFS_LIB=build/var/lib_devu.so SQOBFS_DEV_U=$u timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wire_dense or ragged or unit_sizes or jumbo" > $O/pt_u$u.log 2>&1 || { tail -30 $O/pt_u$u.log; exit 1; }
  echo "U=$u $(tail -1 $O/pt_u$u.log)"
done
for L in devu devkl; do
  SQOBFS_LIB=build/var/lib_$L.so timeout -k 10 300 python -u scripts/dev/unit_sweep.py salamander-1m "16u2 16u3 16u4 16u5 16u6 16u8 14u6 18u6" 7 > $O/$L.txt 2>&1 || { tail -5 $O/$L.txt; exit 1; }
  echo "== $L"; grep ppw $O/$L.txt
done
SQOBFS_LIB=build/var/lib_devu.so timeout -k 10 300 python -u scripts/dev/unit_sweep.py salamander-ragged-4m "28u3 28u4 28u6 26u4 26u6" 5 > $O/ragged.txt 2>&1 || { tail -5 $O/ragged.txt; exit 1; }
grep ppw $O/ragged.txt
