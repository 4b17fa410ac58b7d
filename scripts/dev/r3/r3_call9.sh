#!/bin/bash
# GPU box: whole GPU suite + smoke with the shipped lib, then in-process unit
# sweeps for the one-wave workgroups.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c9; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
sw() { timeout -k 10 300 python -u scripts/dev/unit_sweep.py "$@" > $O/us_$1_${4:-obfuscate}.txt 2>&1 || { tail -5 $O/us_$1_${4:-obfuscate}.txt; exit 1; }; grep ppw $O/us_$1_${4:-obfuscate}.txt | cut -c1-80; }
sw salamander-1m "12 14 16 18 20 24" 5
sw salamander-1m "14 16 18 20" 5 deobfuscate
sw xplus-1m "14 16 18 20 24" 5
sw salamander-ragged-4m "22 24 26 28 30 32 36 40" 5
sw salamander-16m-256psk "20 26 32 40" 3
