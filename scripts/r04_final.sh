#!/usr/bin/env bash
# round 4, final build: GPU suite, smoke, default bench, latency (r04_full.sh),
# then the kernel traces + PMC of configs[1..3] (profile_configs.sh part 1)
# and the device-salt bench line
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/r04_full.sh r04_final || exit 1
timeout -k 10 1000 bash scripts/profile_configs.sh r04f 1 || { echo "profiles rc=$?"; exit 1; }
timeout -k 10 200 python -u bench.py --steps 50 --no-cpu-baseline --device-salt > gpurun_out/r04f/devsalt.json \
  2> gpurun_out/r04f/devsalt.err || { echo "devsalt rc=$?"; tail gpurun_out/r04f/devsalt.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04f/devsalt.json')); r=d['roofline']; print('devsalt', d['value'], r['kernel_avg_us'], r['frac'])"
