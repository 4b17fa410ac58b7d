#!/usr/bin/env bash
# round 4: the whole GPU suite, smoke and the default bench line on one box
# (the driver's round-end sequence), each step under its own time limit
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04_full}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -60 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err \
  || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 sing-quic_amd/bin/lat_bench > $O/lat.json 2> $O/lat.err \
  || { echo "lat_bench rc=$?"; tail $O/lat.err; exit 1; }
cat $O/lat.json
