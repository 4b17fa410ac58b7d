#!/usr/bin/env bash
# round 4: DPP wave reductions (SQ_DPPRED) and device salts under the
# descriptor loads (SQ_EARLYSALT) -- parity of the combined variant, then
# same-process A/Bs (scripts/dev/ab_libs.py)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/ab2
mkdir -p $O
SQOBFS_LIB=build/ab/lib_dp1es1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_scatter.py tests/test_gpu_fuzz.py tests/test_gpu_out_blocks.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/parity_dp1es1.log 2>&1 \
  || { echo "dp1es1 parity rc=$?"; tail -30 $O/parity_dp1es1.log; exit 1; }
tail -1 $O/parity_dp1es1.log
ab() {  # name config direction layout flags libs...
  local name=$1 cfg=$2 dir=$3 lay=$4 fl=$5; shift 5
  timeout -k 10 300 env AB_NOPARITY=${NOPAR:-} AB_OB=$fl AB_LAYOUT=$lay python -u scripts/dev/ab_libs.py \
    $cfg $dir 5 "$@" > $O/$name.txt 2>&1 || { echo "ab $name rc=$?"; tail $O/$name.txt; exit 1; }
  echo "== $name"; grep "median" $O/$name.txt | tail -4
}
P="build/ab/lib_es0.so build/ab/lib_dp1.so"
ab c1_obf salamander-1m obfuscate dense 0 $P
ab c1_deo salamander-1m deobfuscate dense 0 $P
ab ragged_obf salamander-ragged-4m obfuscate dense 0 $P
ab ragged_deo salamander-ragged-4m deobfuscate dense 0 $P
ab ragged_deo_slot16 salamander-ragged-4m deobfuscate slot16 4 $P
ab xplus_obf xplus-1m obfuscate dense 0 $P
ab multi_obf salamander-16m-256psk obfuscate dense 0 $P
S="build/ab/lib_es0.so build/ab/lib_es1.so build/ab/lib_dp1es1.so"
NOPAR=1 ab devsalt_c1 salamander-1m obfuscate dense 2 $S
NOPAR=1 ab devsalt_ragged salamander-ragged-4m obfuscate dense 2 $S
NOPAR=1 ab devsalt_xplus xplus-1m obfuscate dense 2 $S
