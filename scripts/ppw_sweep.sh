#!/bin/bash
# GPU box: kernel time vs unit size (SQOBFS_TUNE_PPW) per config, REPS
# interleaved passes; usage: scripts/ppw_sweep.sh OUTDIR "ppw list" config...
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift; PPWS=$1; shift
mkdir -p $O
for r in $(seq 1 ${REPS:-3}); do
  for c in "$@"; do
    for w in $PPWS; do
      SQOBFS_TUNE_PPW=$w timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --config $c > $O/${c}_p${w}_r$r.json 2> $O/err.txt || { echo "$c ppw $w FAILED"; tail -5 $O/err.txt; exit 1; }
    done
  done
  echo "pass $r done"
done
python - "$O" <<'PY'
import glob, json, os, re, statistics, sys
res = {}
for f in glob.glob(os.path.join(sys.argv[1], "*_p*_r*.json")):
    m = re.match(r"(.*)_p(\d+)_r\d+\.json", os.path.basename(f))
    d = json.load(open(f))
    res.setdefault(m.group(1), {}).setdefault(int(m.group(2)), []).append(
        (d["roofline"]["kernel_avg_us"], d["parity_spot_check"]))
for c, byw in sorted(res.items()):
    print("==", c)
    for w, v in sorted(byw.items()):
        us = [x[0] for x in v]
        print(f"  ppw {w:3d}  median {statistics.median(us):8.1f} us  all {us}  parity {all(x[1] for x in v)}")
PY
