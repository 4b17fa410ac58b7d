#!/usr/bin/env bash
# round 4: GCM regression + kernel trace of the QUIC rates, ragged
# deobfuscate timeline on the shipped build's source (SQ_TIMELINE variant),
# in-process shard lines with the queued mode's warm-up
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04_misc
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_quic_gcm.py tests/test_gpu_quic_obfs.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > $O/gcm_tests.log 2>&1 || { echo "gcm tests rc=$?"; tail -30 $O/gcm_tests.log; exit 1; }
tail -1 $O/gcm_tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/quic_kt -o kt -- \
  python bench.py --quic --no-cpu-baseline --steps 5 --warmup 1 > $O/quic_kt.json 2> $O/quic_kt.log \
  || { echo "quic trace rc=$?"; tail -5 $O/quic_kt.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04_misc/quic_kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:90]:90s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us")
PY
timeout -k 10 300 python -u scripts/dev/gcm_multi_probe.py 5 > $O/gcm_probe.txt 2>&1 \
  || { echo "gcm probe rc=$?"; tail $O/gcm_probe.txt; exit 1; }
cat $O/gcm_probe.txt
for d in deobfuscate obfuscate; do
  SQOBFS_LIB=build/ab/lib_tl.so timeout -k 10 200 python -u scripts/dev/timeline.py salamander-ragged-4m 0 $d \
    > $O/timeline_ragged_$d.json 2> $O/timeline_$d.err || { echo "timeline rc=$?"; tail $O/timeline_$d.err; exit 1; }
  python -c "import json; d=json.load(open('$O/timeline_ragged_$d.json')); print('$d', {k: d[k] for k in list(d)[:12]})" | cut -c1-900
done
for spec in "q:" "i1f1:--inproc 1 --inflight 1" "i1f2:--inproc 1 --inflight 2" "i2f2:--inproc 2 --inflight 2"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 200 python -u bench.py --steps 50 --no-cpu-baseline $a > $O/inproc_$n.json 2> $O/inproc_$n.err \
    || { echo "bench $n rc=$?"; tail $O/inproc_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/inproc_$n.json')); print('$n', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 sing-quic_amd/bin/lat_bench > $O/lat.json 2> $O/lat.err \
  || { echo "lat_bench rc=$?"; tail $O/lat.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04_misc/lat.json"))
for k, v in d.items():
    if k.startswith("pconn_write") or k.startswith("pconn_read"):
        print(k, " | ".join(f"{n}: {x['p50_us']}/{x['p99_us']}" for n, x in v.items()))
PY
