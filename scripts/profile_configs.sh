#!/bin/bash
# GPU box: kernel trace + PMC passes (scripts/profile.sh) of BASELINE configs
# in both directions, then (PART=all or 2) the default bench line and every
# config / direction / layout (scripts/configs.sh).
# usage: scripts/profile_configs.sh TAG [PART: 1 = configs[1..3], 2 = configs[4] + tables, all]
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r3f}; PART=${2:-all}
mkdir -p gpurun_out/$T
case $PART in
  1) CFGS="salamander-1m xplus-1m salamander-ragged-4m" ;;
  2) CFGS="salamander-16m-256psk" ;;
  *) CFGS="salamander-1m xplus-1m salamander-ragged-4m salamander-16m-256psk" ;;
esac
for c in $CFGS; do
  for d in obfuscate deobfuscate; do
    s=$c; [ $d = deobfuscate ] && s=$c-deobfuscate
    timeout -k 10 400 bash scripts/profile.sh $T/$s --config $c --direction $d > gpurun_out/$T.$s.log 2>&1 \
      || { tail -5 gpurun_out/$T.$s.log; exit 1; }
    echo "$s done"
  done
done
[ $PART = 1 ] && exit 0
timeout -k 10 300 python bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err || exit 1
cat gpurun_out/$T/bench_default.json
timeout -k 10 800 bash scripts/configs.sh $T/cfg > gpurun_out/$T/cfg.txt 2>&1 || { tail -20 gpurun_out/$T/cfg.txt; exit 1; }
cat gpurun_out/$T/cfg.txt
