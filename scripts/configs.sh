#!/bin/bash
# GPU box: every BASELINE config x direction, layouts, device salts, and the
# in-process shard mode, with the shipped lib.  usage: scripts/configs.sh OUTDIR
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-cfg}; mkdir -p $O
run() { timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@"; }
for c in salamander-1m xplus-1m salamander-ragged-4m salamander-16m-256psk; do
  for d in obfuscate deobfuscate; do
    run --config $c --direction $d > $O/${c}_$d.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
  done
done
run --layout slot16 > $O/salamander-1m_slot16.json 2>> $O/err.txt || exit 1
run --layout slot16 --direction deobfuscate > $O/salamander-1m_slot16_deobfuscate.json 2>> $O/err.txt || exit 1
run --layout slot2048 > $O/salamander-1m_slot2048.json 2>> $O/err.txt || exit 1
run --layout slot2048 --direction deobfuscate > $O/salamander-1m_slot2048_deobfuscate.json 2>> $O/err.txt || exit 1
run --config salamander-ragged-4m --layout slot16 > $O/salamander-ragged-4m_slot16.json 2>> $O/err.txt || exit 1
run --config salamander-ragged-4m --layout slot16 --direction deobfuscate > $O/salamander-ragged-4m_slot16_deobfuscate.json 2>> $O/err.txt || exit 1
run --layout inplace > $O/salamander-1m_inplace.json 2>> $O/err.txt || exit 1
run --device-salt > $O/salamander-1m_devsalt.json 2>> $O/err.txt || exit 1
run --inproc 2 > $O/salamander-1m_inproc2.json 2>> $O/err.txt || exit 1
run --inproc 1 > $O/salamander-1m_inproc1.json 2>> $O/err.txt || exit 1
python - "$O" <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.load(open(f)); r = d.get("roofline")
    if r is None:
        print(f"{os.path.basename(f)[:-5]:40s} {d['value']:9.1f} GiB/s  {d['ms_per_step']} ms/step")
        continue
    print(f"{os.path.basename(f)[:-5]:40s} {d['value']:9.1f} GiB/s  kernel {r['kernel_avg_us']:8.1f} us  frac {r['frac']:.3f}  parity {d['parity_spot_check']}")
PY
