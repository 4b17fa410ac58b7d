export TMPDIR=/tmp; O=gpurun_out/size; mkdir -p $O
run() { timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@"; }
pr() { python -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$1',d['config']['packets_per_gpu'],r['kernel_avg_us'],r['frac'])"; }
run --config salamander-1m > $O/a.json 2>$O/err || exit 1; pr $O/a.json
run --config salamander-1m --packets 16777216 > $O/b.json 2>>$O/err || exit 1; pr $O/b.json
run --config salamander-16m-256psk --packets 1048576 > $O/c.json 2>>$O/err || exit 1; pr $O/c.json
run --config salamander-16m-256psk > $O/d.json 2>>$O/err || exit 1; pr $O/d.json
run --config salamander-1m --packets 16777216 --direction deobfuscate > $O/e.json 2>>$O/err || exit 1; pr $O/e.json
run --config salamander-16m-256psk --packets 1048576 --direction deobfuscate > $O/f.json 2>>$O/err || exit 1; pr $O/f.json
