export TMPDIR=/tmp
mkdir -p gpurun_out/tl
for v in tl tlp64 tlp16; do
  SQOBFS_LIB=build/var/lib_$v.so SQ_TIMELINE_OUT=gpurun_out/tl/$v.npy timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/tl/$v.json 2>gpurun_out/tl/$v.err || exit 1
  echo "== $v $(python -c "import json;d=json.load(open('gpurun_out/tl/$v.json'));print(d['roofline']['kernel_avg_us'])")"
  python scripts/timeline.py gpurun_out/tl/$v.npy 2847932416
done
