#!/bin/bash
# On the GPU box: bench every BASELINE config and direction with the shipped lib.
export TMPDIR=/tmp
O=gpurun_out/${1:-cfg}; mkdir -p $O
run() { timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@"; }
for c in salamander-1m xplus-1m salamander-ragged-4m salamander-16m-256psk; do
  for d in obfuscate deobfuscate; do
    run --config $c --direction $d > $O/${c}_$d.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
  done
done
run --layout slot16 > $O/salamander-1m_slot16.json 2>> $O/err.txt
run --layout inplace > $O/salamander-1m_inplace.json 2>> $O/err.txt
python - "$O" <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.load(open(f)); r = d["roofline"]
    print(f"{os.path.basename(f)[:-5]:40s} {d['value']:9.1f} GiB/s  kernel {r['kernel_avg_us']:8.1f} us  frac {r['frac']:.3f}  parity {d['parity_spot_check']}")
PY
