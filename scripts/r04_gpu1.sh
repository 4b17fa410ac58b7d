#!/usr/bin/env bash
# round 4, first GPU pass: the new parity / engine tests, the latency bench,
# and the window-load A/B for Salamander deobfuscate (build/ab libraries)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_cpu_path.py tests/test_pconn.py tests/test_gpu_shard.py -m gpu \
  tests/test_gpu_fullsize.py > gpurun_out/r04_tests.log 2>&1 \
  || { echo "tests failed rc=$?"; tail -40 gpurun_out/r04_tests.log; exit 1; }
tail -3 gpurun_out/r04_tests.log
timeout -k 10 300 sing-quic_amd/bin/lat_bench > gpurun_out/r04_lat.json 2> gpurun_out/r04_lat.err \
  || { echo "lat_bench rc=$?"; tail gpurun_out/r04_lat.err; exit 1; }
echo lat ok
L="build/ab/lib_base.so build/ab/lib_ws1p.so build/ab/lib_ws2.so build/ab/lib_ws2p.so"
ab() {  # name config direction [env]
  local name=$1; shift
  timeout -k 10 300 env "$@" python -u scripts/dev/ab_libs.py $CFG $DIR 5 $L \
    > gpurun_out/ab/$name.txt 2>&1 || { echo "ab $name rc=$?"; tail gpurun_out/ab/$name.txt; exit 1; }
  tail -6 gpurun_out/ab/$name.txt
}
CFG=salamander-ragged-4m DIR=deobfuscate ab ragged_deo_dense AB_LAYOUT=dense
CFG=salamander-ragged-4m DIR=deobfuscate ab ragged_deo_slot16 AB_LAYOUT=slot16
CFG=salamander-1m DIR=deobfuscate ab c1_deo AB_LAYOUT=dense
CFG=salamander-1m DIR=obfuscate ab c1_obf AB_LAYOUT=dense
CFG=salamander-ragged-4m DIR=obfuscate ab ragged_obf_dense AB_LAYOUT=dense
CFG=xplus-1m DIR=deobfuscate ab xplus_deo AB_LAYOUT=dense
