#!/bin/bash
# On the GPU box: per BASELINE config, one rocprofv3 kernel-trace pass and two
# PMC passes (FETCH_SIZE, WRITE_SIZE; never combined with tracing), each under
# its own time limit.  Summaries land in gpurun_out/$TAG/<config>/.
# usage: scripts/profile_all.sh TAG [config ...]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-prof}; shift
CONFIGS=${*:-salamander-1m xplus-1m salamander-ragged-4m salamander-16m-256psk}
for c in $CONFIGS; do
  O=gpurun_out/$TAG/$c; mkdir -p $O
  B="python bench.py --config $c --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- $B --steps 20 --warmup 3 > $O/bench_kt.json 2> $O/kt.log || { tail -5 $O/kt.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p1 -o p -- $B --steps 5 --warmup 1 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p2 -o p -- $B --steps 5 --warmup 1 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
  python scripts/pmc_summary.py $O > /dev/null || exit 1
  find $O/kt -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
  echo "$c: $(grep obfs_kernel $O/kernel_stats.csv | cut -d, -f1-5 | head -2 | tr '\n' ' ')"
  python -c "import json,sys; d=json.load(open('$O/summary.json')); print('  hbm bytes/launch', d.get('hbm_bytes_per_launch'))"
done
