#!/bin/bash
# On the GPU box: collect PMC counter passes for bench.py (one counter group per
# pass; never combined with tracing).  usage: scripts/pmc.sh TAG [bench args]
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/pmc_$TAG; mkdir -p $O
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum" \
           "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" \
           "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_LEVEL_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $O/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -5 $O/p$i.log; exit 1; }
done
python scripts/pmc_summary.py $O
