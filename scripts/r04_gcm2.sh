#!/usr/bin/env bash
# round 4: key-grouped GCM (steps of one key) -- tests, in-process probe by key layout, rates
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04_gcm2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_quic_gcm.py tests/test_gpu_quic_obfs.py tests/test_gpu_quic.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "gcm tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/dev/gcm_multi_probe.py 5 > $O/gcm_probe.txt 2>&1 \
  || { echo "gcm probe rc=$?"; tail $O/gcm_probe.txt; exit 1; }
cat $O/gcm_probe.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/quic_kt -o kt -- \
  python bench.py --quic --no-cpu-baseline --steps 5 --warmup 1 > $O/quic_kt.json 2> $O/quic_kt.log \
  || { echo "quic trace rc=$?"; tail -5 $O/quic_kt.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04_gcm2/quic_kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "sq::" in r["Name"]:
        print(f"{r['Name'][:80]:80s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us")
PY
