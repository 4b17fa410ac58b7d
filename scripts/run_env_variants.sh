#!/bin/bash
# On the GPU box: bench the in-tree libsqobfs.so under several environment
# settings (tuning knobs such as SQOBFS_TILE), REPS interleaved passes,
# median kernel us per setting.
# usage: REPS=3 scripts/run_env_variants.sh TAG "name:VAR=1 VAR2=2" ... -- [bench args]
export TMPDIR=/tmp
O=gpurun_out/${1:-envvar}; shift; mkdir -p $O
specs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do specs+=("$1"); shift; done
[ "$1" = "--" ] && shift
REPS=${REPS:-3}
for r in $(seq 1 $REPS); do
  for spec in "${specs[@]}"; do
    n=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > $O/${n}_r$r.json 2> $O/$n.err || { echo "$n FAILED"; tail -3 $O/$n.err; exit 1; }
  done
done
python - "$O" <<'PY'
import glob, json, os, statistics, sys
o = sys.argv[1]
res = {}
for f in sorted(glob.glob(os.path.join(o, "*_r*.json"))):
    name = os.path.basename(f).rsplit("_r", 1)[0]
    d = json.load(open(f))
    res.setdefault(name, []).append((d["ms_per_step"] * 1e3, d["roofline"]["kernel_avg_us"], d["parity_spot_check"]))
for name, v in sorted(res.items(), key=lambda kv: statistics.median(x[0] for x in kv[1])):
    us = [round(x[0], 1) for x in v]
    print(f"{name:16s} step median {statistics.median(us):8.1f} us  all {us}  parity {all(x[2] for x in v)}")
PY
