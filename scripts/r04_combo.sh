#!/usr/bin/env bash
# round 4: the whole GPU suite, then the grouped-GCM probe and QUIC kernel
# trace, then the latency tool (measured routing)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_combo}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
grep -h "routing:\|break-even" $O/gpu_tests.log || true
timeout -k 10 300 python -u scripts/dev/gcm_multi_probe.py 5 > $O/gcm_probe.txt 2>&1 \
  || { echo "gcm probe rc=$?"; tail $O/gcm_probe.txt; exit 1; }
cat $O/gcm_probe.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/quic_kt -o kt -- \
  python bench.py --quic --no-cpu-baseline --steps 5 --warmup 1 > $O/quic_kt.json 2> $O/quic_kt.log \
  || { echo "quic trace rc=$?"; tail -5 $O/quic_kt.log; exit 1; }
python - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/quic_kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "sq::" in r["Name"]:
        print(f"{r['Name'][:80]:80s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us")
PY
timeout -k 10 300 sing-quic_amd/bin/lat_bench > $O/lat.json 2> $O/lat.err \
  || { echo "lat_bench rc=$?"; tail $O/lat.err; exit 1; }
python - "$O" <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + "/lat.json"))
for k, v in d.items():
    if k.startswith("pconn_write") or k.startswith("pconn_read"):
        print(k, " | ".join(f"{n}: {x['p50_us']}/{x['p99_us']}" for n, x in v.items()))
    elif "stats" in k:
        print(k, v)
PY
