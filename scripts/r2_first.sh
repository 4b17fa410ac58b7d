set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2a
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/pytest.log 2>&1 && \
timeout -k 10 180 python bench.py > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err
