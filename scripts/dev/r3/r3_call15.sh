#!/bin/bash
# GPU box: QUIC AES-128-GCM kernel packets per wave / waves per workgroup.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c15; mkdir -p $O
for L in g32 g24 g24b; do
  SQOBFS_LIB=build/var/lib_$L.so timeout -k 10 300 python -u -m pytest tests/test_gpu_quic_gcm.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_$L.log 2>&1 || { tail -30 $O/pt_$L.log; exit 1; }
  echo "$L $(tail -1 $O/pt_$L.log)"
done
for r in 1 2 3; do
  for L in g16 g32 g24 g24b; do
    SQOBFS_LIB=build/var/lib_$L.so timeout -k 10 120 python scripts/quic_prof.py 1 20 2>&1 | grep -E "seal|ok|rror" | tr '\n' ' ' | sed "s/^/$L r$r /" | cut -c1-110; echo
  done
done
