#!/bin/bash
# GPU box: kernel trace and VALU/LDS PMC passes of bench.py --quic (QUIC kernels).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
  python bench.py --quic --no-cpu-baseline --steps 5 --warmup 1 > $O/kt.json 2> $O/kt.log \
  || { tail -5 $O/kt.log; exit 1; }
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p -- \
    python bench.py --quic --no-cpu-baseline --steps 3 --warmup 1 > $O/p$i.log 2>&1 \
    || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python scripts/quic_pmc_summary.py $O
