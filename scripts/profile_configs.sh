#!/bin/bash
# GPU box: kernel trace + PMC passes (scripts/profile.sh) of every BASELINE
# config, both directions, then the default bench line and every config /
# direction / layout (scripts/configs.sh).  usage: scripts/profile_configs.sh TAG
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r3f}
mkdir -p gpurun_out/$T
for c in salamander-1m xplus-1m salamander-ragged-4m salamander-16m-256psk; do
  for d in obfuscate deobfuscate; do
    s=$c; [ $d = deobfuscate ] && s=$c-deobfuscate
    timeout -k 10 400 bash scripts/profile.sh $T/$s --config $c --direction $d > gpurun_out/$T.$s.log 2>&1 \
      || { tail -5 gpurun_out/$T.$s.log; exit 1; }
  done
done
timeout -k 10 300 python bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err || exit 1
cat gpurun_out/$T/bench_default.json
timeout -k 10 800 bash scripts/configs.sh $T/cfg > gpurun_out/$T/cfg.txt 2>&1 || { tail -20 gpurun_out/$T/cfg.txt; exit 1; }
cat gpurun_out/$T/cfg.txt
