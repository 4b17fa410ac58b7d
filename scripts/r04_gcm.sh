#!/usr/bin/env bash
# round 4: key-grouped multi-key AES-128-GCM -- its tests, then the QUIC rates
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04_gcm
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_quic_gcm.py tests/test_gpu_quic_obfs.py -m gpu -x -v \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "gcm tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --quic --no-cpu-baseline --steps 10 > $O/quic.json 2> $O/quic.err \
  || { echo "quic bench rc=$?"; tail $O/quic.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04_gcm/quic.json"))["quic"]
for s, v in d.items():
    print(s, json.dumps({k: v[k] for k in v if "us" in k or "GiB" in k or "multi" in k})[:900])
PY
