#!/bin/bash
# On the GPU box: QUIC kernel trace + bench line (both suites) into
# gpurun_out/quic_final/ (copied to profiles/r01/quic/ by collect_profiles.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final/quic; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python scripts/quic_prof.py 1 6 > $O/kt_gcm.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt2 -o kt -- python scripts/quic_prof.py 0 6 > $O/kt_chacha.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --quic --steps 10 > $O/bench_quic.json 2> $O/bench.err || exit 1
cat $O/kt_gcm.log $O/kt_chacha.log
