#!/bin/bash
# GPU box: QUIC ChaCha20-Poly1305 kernel workgroup size (4 / 2 / 1 waves):
# parity of each build, then interleaved timing.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c13; mkdir -p $O
for L in q128 q64; do
  SQOBFS_LIB=build/var/lib_$L.so timeout -k 10 300 python -u -m pytest tests/test_gpu_quic.py tests/test_gpu_quic_obfs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_$L.log 2>&1 || { tail -30 $O/pt_$L.log; exit 1; }
  echo "$L $(tail -1 $O/pt_$L.log)"
done
for r in 1 2 3; do
  for L in q256 q128 q64; do
    SQOBFS_LIB=build/var/lib_$L.so timeout -k 10 120 python scripts/quic_prof.py 0 40 2>&1 | grep -E "seal|ok|rror" | tr '\n' ' ' | sed "s/^/$L r$r /"; echo
  done
done
