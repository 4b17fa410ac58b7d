#!/bin/bash
# GPU box: parity then same-process timing of kernel variants built by
# scripts/variants.sh into build/ab (lib_base.so = the shipped flags).
#   parity: the GPU parity files (golden vectors, oracle, fuzz, scatter,
#           slotted layouts, device salts) against each variant
#   timing: scripts/dev/ragged_split.py (base vs the variants, both
#           directions) and device-salt / host-salt ab_libs runs
# usage: scripts/dev/variant_ab.sh OUTDIR "variant ..." [ROUNDS]
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-vab}; V=$2; R=${3:-5}
mkdir -p $O
for v in $V; do
  SQOBFS_LIB=build/ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_fuzz.py tests/test_gpu_scatter.py tests/test_gpu_out_blocks.py \
    tests/test_gpu_slot_staging.py tests/test_gpu_cpu_path.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > $O/parity_$v.log 2>&1 \
    || { echo "parity $v failed"; tail -30 $O/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $O/parity_$v.log)"
done
L="build/ab/lib_base.so"
for v in $V; do L="$L build/ab/lib_$v.so"; done
for d in obfuscate deobfuscate; do
  timeout -k 10 500 python -u scripts/dev/ragged_split.py $d $R $L > $O/split_$d.txt 2>&1 \
    || { echo "split $d failed"; tail -5 $O/split_$d.txt; exit 1; }
done
grep -h median $O/split_*.txt
# device salts: the variants side by side, and host vs device salts per lib
for c in salamander-1m salamander-ragged-4m xplus-1m; do
  timeout -k 10 300 env AB_NOPARITY=1 AB_OB=2 python -u scripts/dev/ab_libs.py $c obfuscate $R $L \
    > $O/devsalt_$c.txt 2>&1 || { echo "devsalt $c failed"; tail -5 $O/devsalt_$c.txt; exit 1; }
  tail -n $(( $(echo $V | wc -w) + 1 )) $O/devsalt_$c.txt
  for lib in $L; do
    n=$(basename $lib .so)
    timeout -k 10 300 env AB_NOPARITY=1 AB_FLAGS=0,2 python -u scripts/dev/ab_libs.py $c obfuscate $R \
      $lib > $O/hostdev_${c}_$n.txt 2>&1 || { echo "hostdev $c $n failed"; exit 1; }
    tail -2 $O/hostdev_${c}_$n.txt
  done
done
