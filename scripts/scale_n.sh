#!/bin/bash
# GPU box: kernel time vs batch size (fixed per-launch overhead: start-up and drain)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$1
for n in 262144 1048576 4194304 8388608; do
  timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --packets $n > gpurun_out/$1/n$n.json 2> gpurun_out/$1/n$n.err || { tail -3 gpurun_out/$1/n$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/$1/n$n.json'));r=d['roofline'];print($n, r['kernel_avg_us'], round(r['kernel_avg_us']*1048576/$n,1), r['frac'])"
done
