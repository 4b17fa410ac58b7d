#!/bin/bash
# On the GPU box: time every build/var/lib_*.so on the QUIC kernels
# (scripts/quic_prof.py: 1M x 1350 B seal + open), REPS interleaved passes.
# usage: scripts/quic_variants.sh SUITE [REPS]
export TMPDIR=/tmp
S=${1:-1}; REPS=${2:-2}
for r in $(seq 1 $REPS); do
  for L in build/var/lib_*.so; do
    SQOBFS_LIB=$L timeout -k 10 120 python scripts/quic_prof.py $S 6 2>&1 | grep -E "seal|Error|error" || { echo "$L FAILED"; exit 1; }
  done
done
