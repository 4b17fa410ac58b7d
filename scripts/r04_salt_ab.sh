#!/usr/bin/env bash
# round 4: device salts computed under the descriptor loads (SQ_EARLYSALT) --
# parity of the variant (device-salt and engine tests), then the same-process
# A/B on device-salted obfuscate launches
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/ab_salt
mkdir -p $O
SQOBFS_LIB=build/ab/lib_es1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_cpu_path.py -m gpu -x -q --timeout 120 --timeout-method thread -k "salt" \
  > $O/parity_es1.log 2>&1 || { echo "es1 parity rc=$?"; tail -30 $O/parity_es1.log; exit 1; }
tail -1 $O/parity_es1.log
L="build/ab/lib_es0.so build/ab/lib_es1.so"
ab() {  # name config layout flags
  timeout -k 10 300 env AB_NOPARITY=1 AB_OB=${4:-2} AB_LAYOUT=$3 python -u scripts/dev/ab_libs.py $2 obfuscate 5 $L \
    > $O/$1.txt 2>&1 || { echo "ab $1 rc=$?"; tail $O/$1.txt; exit 1; }
  echo "== $1"; tail -3 $O/$1.txt
}
ab devsalt_c1 salamander-1m dense
ab devsalt_ragged salamander-ragged-4m dense
ab devsalt_xplus xplus-1m dense
ab devsalt_c1_slot16 salamander-1m slot16 6
