#!/bin/bash
# GPU box: waves per workgroup (1 / 2 / 4) per kernel, in one process per
# config (dev build), plus parity of the shipped lib's new launch shapes.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c11; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
echo "shipped $(tail -1 $O/pt.log)"
sw() { SQOBFS_LIB=build/var/lib_dev.so timeout -k 10 300 python -u scripts/dev/unit_sweep.py "$@" > $O/$1_${4:-obfuscate}.txt 2>&1 || { tail -5 $O/$1_${4:-obfuscate}.txt; exit 1; }; grep ppw $O/$1_${4:-obfuscate}.txt | cut -c1-84; }
sw salamander-1m "16w1 16w2 16w4 18w1 18w4" 5
sw salamander-1m "16w1 16w2 16w4" 5 deobfuscate
sw xplus-1m "18w1 18w2 18w4 16w1 16w4" 5
sw xplus-1m "18w1 18w2 18w4" 5 deobfuscate
sw salamander-ragged-4m "28w1 28w2 28w4" 5
sw salamander-ragged-4m "28w1 28w2 28w4" 5 deobfuscate
sw salamander-16m-256psk "26w1 26w2 26w4" 3
sw salamander-16m-256psk "26w1 26w2 26w4" 3 deobfuscate
