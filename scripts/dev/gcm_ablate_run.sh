#!/bin/bash
# GPU box: kernel time of each build of scripts/dev/gcm_ablate.py (AES-128-GCM
# seal / open of 1M x 1,361-B packets, scripts/quic_prof.py), one process per
# build, then a table.  usage: scripts/dev/gcm_ablate_run.sh OUTDIR
# (SUITE=0: the ChaCha20-Poly1305 kernels instead)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for v in $(ls build/ablate); do
  SQOBFS_LIB=$PWD/build/ablate/$v/libsqobfs.so timeout -k 10 120 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $O/$v -o kt -- python3 scripts/quic_prof.py ${SUITE:-1} 6 > $O/$v.log 2>&1 \
    || { tail -5 $O/$v.log; exit 1; }
done
python3 - "$O" <<'PY' | tee $O/summary.txt
import csv, glob, os, sys
o = sys.argv[1]
for d in sorted(glob.glob(f"{o}/*/")):
    f = glob.glob(f"{d}**/*kernel_stats.csv", recursive=True)
    if not f:
        continue
    r = {x["Name"]: float(x["AverageNs"]) / 1e3 for x in csv.DictReader(open(f[0])) if "quic_" in x["Name"] and "group" not in x["Name"]}
    print(os.path.basename(d.rstrip("/")), {k.split("<")[1].split(">")[0]: round(v, 1) for k, v in r.items()})
PY
