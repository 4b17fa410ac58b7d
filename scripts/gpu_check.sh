#!/bin/bash
# GPU-box check: parity tests, smoke, bench (+ optional rocprofv3 passes).
# usage: scripts/gpu_check.sh TAG [tests|notests] [prof|noprof] [extra bench args...]
set -o pipefail
TAG=${1:-run}; TESTS=${2:-tests}; PROF=${3:-noprof}; shift 3 2>/dev/null
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
if [ "$TESTS" = tests ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x -rf > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-seconds 1 "$@" > $O/bench.json 2> $O/bench.err || { cat $O/bench.err | tail -20; exit 1; }
cat $O/bench.json
if [ "$PROF" = prof ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > $O/kt.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $O/fetch.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $O/write.log 2>&1 || exit $?
  grep obfs_kernel $O/kt/kt_kernel_stats.csv | cut -c1-200
fi
