#!/bin/bash
# Dev (GPU box): run the ASan builds of scripts/dev/asan_build.sh.  Leak
# checking stays off (the HIP runtime keeps allocations to process exit);
# protect_shadow_gap=0 leaves the address range the GPU runtime maps.
cd "$(dirname "$0")/../.."
O=gpurun_out/asan; mkdir -p $O
export ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1:abort_on_error=0
for t in test_cgo_sequence test_pconn test_packet_conn lat_bench; do
  timeout -k 10 300 build/asan/$t > $O/$t.log 2>&1; rc=$?
  echo "$t rc=$rc"; tail -4 $O/$t.log
  grep -c "ERROR: AddressSanitizer" $O/$t.log
done
