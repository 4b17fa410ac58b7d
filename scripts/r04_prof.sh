#!/usr/bin/env bash
# round 4 profiles: kernel traces + PMC of the BASELINE configs
# (scripts/profile_configs.sh, part 1 or 2), then the in-process multi-context
# bench lines against queued launches (part 1) or the layout table (part 2)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
PART=${1:-1}
timeout -k 10 1000 bash scripts/profile_configs.sh r04 $PART || { echo "profiles rc=$?"; exit 1; }
if [ "$PART" = 1 ]; then
  O=gpurun_out/r04/inproc
  mkdir -p $O
  for spec in "q:" "i1f1:--inproc 1 --inflight 1" "i1f2:--inproc 1 --inflight 2" \
              "i2f2:--inproc 2 --inflight 2" "q2:"; do
    n=${spec%%:*}; a=${spec#*:}
    timeout -k 10 200 python -u bench.py --steps 50 --no-cpu-baseline $a > $O/$n.json 2> $O/$n.err \
      || { echo "bench $n rc=$?"; tail $O/$n.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'])"
  done
fi
