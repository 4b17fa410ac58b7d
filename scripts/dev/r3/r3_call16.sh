#!/bin/bash
# GPU box: whole GPU suite + smoke, QUIC PMC (VALU roofline) and the QUIC bench.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c16; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash scripts/r2_quic_pmc.sh r3c16/qp > $O/qp.log 2>&1 || { tail -10 $O/qp.log; exit 1; }
tail -8 $O/qp.log
