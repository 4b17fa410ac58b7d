#!/bin/bash
# GPU box: parity of the salt-word-specialised hash builds, then in-process
# timing: 4 vs 3 waves per SIMD (LDS pad) at several unit sizes.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c7; mkdir -p $O
for L in kw4 kw3; do
  SQOBFS_LIB=build/var/lib_$L.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_$L.log 2>&1 || { tail -30 $O/pt_$L.log; exit 1; }
  echo "$L $(tail -1 $O/pt_$L.log)"
done
sw() { L=$1; shift; SQOBFS_LIB=build/var/lib_$L.so timeout -k 10 300 python -u scripts/dev/unit_sweep.py "$@" > $O/${L}_$1_${4:-obf}.txt 2>&1 || { tail -5 $O/${L}_$1_${4:-obf}.txt; exit 1; }; echo "== $L"; grep ppw $O/${L}_$1_${4:-obf}.txt; }
sw kw4 salamander-1m "16 16u4l800 12 14 18 20 24 16u2 16u3" 5
sw kw4 salamander-1m "16 16u4l800 14 20" 5 deobfuscate
sw kw4 salamander-ragged-4m "28 28u4l800 24 32 36" 5
sw kw3 salamander-1m "16 14 18" 5
sw old salamander-1m "16 14 18" 5
