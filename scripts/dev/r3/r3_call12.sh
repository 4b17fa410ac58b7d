#!/bin/bash
# GPU box: full GPU suite + smoke (shipped lib), unit-size sweeps at 2-wave
# workgroups, then profiles of every config and the config table.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c12; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
sw() { timeout -k 10 300 python -u scripts/dev/unit_sweep.py "$@" > $O/us_$1_${4:-obfuscate}.txt 2>&1 || { tail -5 $O/us_$1_${4:-obfuscate}.txt; exit 1; }; grep ppw $O/us_$1_${4:-obfuscate}.txt | cut -c1-80; }
sw salamander-1m "14 16 18 20" 5
sw xplus-1m "14 16 18 20" 5
sw salamander-ragged-4m "24 26 28 30 32" 5
bash scripts/r3_final.sh r3g
