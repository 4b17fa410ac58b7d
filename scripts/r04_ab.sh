#!/usr/bin/env bash
# round 4: window-load variants of the obfuscation kernel (build/ab, made by
# scripts/variants.sh) -- parity of each on the core parity file, then the
# same-process A/B per config / direction / layout
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${AB_OUT:-ab}
mkdir -p $O
L=${AB_LIBS:-"build/ab/lib_base.so build/ab/lib_wb1.so build/ab/lib_wb2.so"}
for lib in $L; do
  n=$(basename $lib .so)
  [ "$n" = lib_base ] && continue
  SQOBFS_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scatter.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/parity_$n.log 2>&1 \
    || { echo "$n parity rc=$?"; tail -30 $O/parity_$n.log; exit 1; }
  echo "$n $(tail -1 $O/parity_$n.log)"
done
ab() {  # name config direction layout
  timeout -k 10 300 env AB_LAYOUT=$4 python -u scripts/dev/ab_libs.py $2 $3 ${AB_ROUNDS:-5} $L \
    > $O/$1.txt 2>&1 || { echo "ab $1 rc=$?"; tail $O/$1.txt; exit 1; }
  echo "== $1"; tail -8 $O/$1.txt
}
ab ragged_deo_dense salamander-ragged-4m deobfuscate dense
ab ragged_deo_slot16 salamander-ragged-4m deobfuscate slot16
ab c1_deo salamander-1m deobfuscate dense
ab c1_obf salamander-1m obfuscate dense
ab ragged_obf_dense salamander-ragged-4m obfuscate dense
ab xplus_deo xplus-1m deobfuscate dense
ab xplus_obf xplus-1m obfuscate dense
ab multi_obf salamander-16m-256psk obfuscate dense
# the image windows' share of slot2048 obfuscate (SQ_ABLATE=8 skips their
# loads: timing only, its output is wrong)
L="build/ab/lib_base.so build/ab/lib_abl8.so"
AB_NOPARITY=1 AB_OB=8 ab slot2048_obf_abl8 salamander-1m obfuscate slot2048
AB_NOPARITY=1 ab c1_obf_abl8 salamander-1m obfuscate dense
