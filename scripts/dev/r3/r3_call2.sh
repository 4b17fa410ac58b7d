#!/bin/bash
# GPU box: in-process unit-size sweeps (warm) per config and direction.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c2; mkdir -p $O
sw() { timeout -k 10 300 python -u scripts/dev/unit_sweep.py "$@" > $O/us_$1_${4:-obfuscate}.txt 2>&1 || { tail -5 $O/us_$1_${4:-obfuscate}.txt; exit 1; }; grep ppw $O/us_$1_${4:-obfuscate}.txt; }
sw salamander-1m "10 12 14 16 18 20 22 26" 5
sw salamander-1m "10 12 14 16 18 20 26 32" 5 deobfuscate
sw xplus-1m "10 12 14 16 18 20 26" 5
sw salamander-ragged-4m "18 20 22 24 26 28 30 32" 5
sw salamander-16m-256psk "12 14 16 18 20 26 32" 3
