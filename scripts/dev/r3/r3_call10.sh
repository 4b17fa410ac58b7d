#!/bin/bash
# GPU box: one-wave vs four-wave workgroups on the multi-PSK and XPlus
# configs and both directions, interleaved processes.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c10; mkdir -p $O
for r in 1 2; do
  for L in b256 b64; do
    for spec in "salamander-16m-256psk|26|3|obfuscate" "salamander-16m-256psk|26|3|deobfuscate" "xplus-1m|18|3|obfuscate" "salamander-1m|16|3|deobfuscate" "salamander-ragged-4m|28|3|deobfuscate"; do
      IFS='|' read c w n d <<< "$spec"
      SQOBFS_LIB=build/var/lib_$L.so timeout -k 10 300 python -u scripts/dev/unit_sweep.py $c "$w" $n $d > $O/${L}_${c}_${d}_r$r.txt 2>&1 || { tail -5 $O/${L}_${c}_${d}_r$r.txt; exit 1; }
      grep ppw $O/${L}_${c}_${d}_r$r.txt | sed "s/^/$L r$r /" | cut -c1-90
    done
  done
done
