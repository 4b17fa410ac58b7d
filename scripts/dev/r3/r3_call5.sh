#!/bin/bash
# GPU box: lane-pair key parity (unit sizes <= 31) and in-process A/B timing.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c5; mkdir -p $O
SQOBFS_DEV_KEY_LANES=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pair_test.log 2>&1 || { tail -30 $O/pair_test.log; exit 1; }
tail -1 $O/pair_test.log
sw() { timeout -k 10 300 python -u scripts/dev/unit_sweep.py "$@" > $O/ab_$1_${4:-obfuscate}.txt 2>&1 || { tail -5 $O/ab_$1_${4:-obfuscate}.txt; exit 1; }; grep ppw $O/ab_$1_${4:-obfuscate}.txt; }
sw salamander-1m "14 14p 16 16p 12p" 7
sw salamander-1m "14 14p" 7 deobfuscate
sw salamander-ragged-4m "26 26p 24p" 5
sw salamander-16m-256psk "26 26p" 3
