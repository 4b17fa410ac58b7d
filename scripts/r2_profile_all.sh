#!/bin/bash
# GPU box: r2_profile.sh (kernel trace + PMC passes) for every BASELINE config
# (obfuscate) plus configs[1] deobfuscate, then the default bench line.
cd $GRAFT_REPO_ROOT
T=${1:-r2p}
for c in salamander-1m xplus-1m salamander-ragged-4m salamander-16m-256psk; do
  bash scripts/r2_profile.sh $T/$c --config $c > gpurun_out/$T.$c.log 2>&1 || { tail -5 gpurun_out/$T.$c.log; exit 1; }
done
bash scripts/r2_profile.sh $T/salamander-1m-deobfuscate --direction deobfuscate > gpurun_out/$T.deo.log 2>&1 || { tail -5 gpurun_out/$T.deo.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err || exit 1
cat gpurun_out/$T/bench_default.json
