#!/bin/bash
# GPU box: in-process unit-size sweeps, deobfuscate direction.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c4; mkdir -p $O
sw() { timeout -k 10 300 python -u scripts/dev/unit_sweep.py "$@" > $O/us_$1_${4:-obfuscate}.txt 2>&1 || { tail -5 $O/us_$1_${4:-obfuscate}.txt; exit 1; }; grep ppw $O/us_$1_${4:-obfuscate}.txt; }
sw salamander-ragged-4m "20 24 26 28 32 40 48" 5 deobfuscate
sw xplus-1m "12 14 16 18 20 26" 5 deobfuscate
sw salamander-16m-256psk "20 26 32 40 48 62" 3 deobfuscate
sw salamander-16m-256psk "32 40 48 62" 3
