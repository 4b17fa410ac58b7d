#!/usr/bin/env bash
# round 4: unit-size sweeps of the deobfuscate kernels (one library, one
# process, interleaved rounds; scripts/dev/ab_libs.py AB_PPWS)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
sweep() {  # name config direction layout ppws [lib]
  local lib=${6:-sing-quic_amd/libsqobfs.so}
  timeout -k 10 300 env AB_LAYOUT=$4 AB_PPWS=$5 python -u scripts/dev/ab_libs.py $2 $3 5 $lib \
    > gpurun_out/ab/$1.txt 2>&1 || { echo "sweep $1 rc=$?"; tail gpurun_out/ab/$1.txt; exit 1; }
  tail -8 gpurun_out/ab/$1.txt
}
sweep unit_ragged_deo_dense salamander-ragged-4m deobfuscate dense 24,28,32,36,40,48
sweep unit_ragged_deo_slot16 salamander-ragged-4m deobfuscate slot16 24,28,32,36,40,48
sweep unit_c1_deo salamander-1m deobfuscate dense 14,16,20,24,28
sweep unit_ragged_obf_slot16 salamander-ragged-4m obfuscate slot16 24,28,32,36,40
