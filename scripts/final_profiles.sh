set -o pipefail
export TMPDIR=/tmp
bash scripts/profile_all.sh final > gpurun_out/prof_final.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/final/bench_default.json 2> gpurun_out/final/bench_default.err || exit 1
mkdir -p gpurun_out/final/quic
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/quic/kt -o kt -- python bench.py --quic --no-cpu-baseline > gpurun_out/final/quic/bench_quic_kt.json 2> gpurun_out/final/quic/kt.log || exit 1
timeout -k 10 300 python bench.py --quic > gpurun_out/final/quic/bench_quic.json 2> gpurun_out/final/quic/bench.err || exit 1
cat gpurun_out/prof_final.log; cat gpurun_out/final/bench_default.json; cat gpurun_out/final/quic/bench_quic.json
