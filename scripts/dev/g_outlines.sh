export TMPDIR=/tmp; O=gpurun_out/s5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 bash scripts/profile.sh s5/slot2048_obfuscate --layout slot2048 > $O/p_obf.log 2>&1 || { tail $O/p_obf.log; exit 1; }
timeout -k 10 400 bash scripts/profile.sh s5/slot2048_deobfuscate --layout slot2048 --direction deobfuscate > $O/p_deo.log 2>&1 || { tail $O/p_deo.log; exit 1; }
for d in obfuscate deobfuscate; do python -c "import json,sys;d=json.load(open('$O/slot2048_$d/kt.json'));r=d['roofline'];print('$d',r['kernel_avg_us'],r['frac'],d['config']['batch_flags'])"; done
