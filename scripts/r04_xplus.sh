#!/usr/bin/env bash
# round 4: the XPlus configs' kernel traces + PMC passes after the XPlus unit
# rule (16 packets per wave), then the GPU suite, smoke and the default bench
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 400 bash scripts/profile.sh r04x/xplus-1m --config xplus-1m --direction obfuscate \
  > gpurun_out/r04x.xplus-1m.log 2>&1 || { tail -5 gpurun_out/r04x.xplus-1m.log; exit 1; }
timeout -k 10 400 bash scripts/profile.sh r04x/xplus-1m-deobfuscate --config xplus-1m --direction deobfuscate \
  > gpurun_out/r04x.xplus-1m-deobfuscate.log 2>&1 || { tail -5 gpurun_out/r04x.xplus-1m-deobfuscate.log; exit 1; }
echo "xplus profiles done"
bash scripts/r04_full.sh r04_full5
