#!/bin/bash
# On the GPU box: bench every build/var/lib_*.so, REPS interleaved passes,
# report median kernel us (parity from the last pass).
export TMPDIR=/tmp
O=gpurun_out/${1:-var}; shift; mkdir -p $O
REPS=${REPS:-3}
for r in $(seq 1 $REPS); do
  for L in build/var/lib_*.so; do
    n=$(basename $L .so)
    SQOBFS_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > $O/${n}_r$r.json 2> $O/$n.err || { echo "$n FAILED"; tail -3 $O/$n.err; exit 1; }
  done
done
python - "$O" <<'PY'
import glob, json, os, statistics, sys
o = sys.argv[1]
res = {}
for f in sorted(glob.glob(os.path.join(o, "*_r*.json"))):
    name = os.path.basename(f).rsplit("_r", 1)[0]
    d = json.load(open(f))
    res.setdefault(name, []).append((d["roofline"]["kernel_avg_us"], d["parity_spot_check"]))
for name, v in sorted(res.items(), key=lambda kv: statistics.median(x[0] for x in kv[1])):
    us = [x[0] for x in v]
    print(f"{name:16s} median {statistics.median(us):8.1f} us  all {us}  parity {all(x[1] for x in v)}")
PY
