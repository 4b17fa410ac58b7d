#!/usr/bin/env bash
# round 4: the GPU fuzz test, then the QUIC kernels' PMC (VALU rate of the
# grouped multi-key GCM kernels) -- scripts/quic_pmc.sh
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/fuzz.log 2>&1 || { echo "fuzz rc=$?"; tail -30 gpurun_out/fuzz.log; exit 1; }
tail -1 gpurun_out/fuzz.log
timeout -k 10 900 bash scripts/quic_pmc.sh r04_quic || { echo "quic pmc failed"; exit 1; }
