export TMPDIR=/tmp; O=gpurun_out/sh1; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "hot_bounds or multi_psk or long_and_empty" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for d in obfuscate deobfuscate; do
  AB_KR=2 timeout -k 10 500 python scripts/dev/ab_libs.py salamander-16m-256psk $d 4 build/var/lib_noshort.so build/var/lib_short.so > $O/ab_$d.txt 2>&1 || { tail -5 $O/ab_$d.txt; exit 1; }
  grep median $O/ab_$d.txt | grep -v instance
done
for d in deobfuscate obfuscate; do
  AB_PPWS=14,16,18,20,23 timeout -k 10 500 python scripts/dev/ab_libs.py salamander-16m-256psk $d 4 build/var/lib_short.so > $O/ppw_$d.txt 2>&1 || { tail -5 $O/ppw_$d.txt; exit 1; }
  grep median $O/ppw_$d.txt | grep -v instance
done
for cd in salamander-16m-256psk:deobfuscate salamander-16m-256psk:obfuscate salamander-1m:obfuscate; do
  c=${cd%%:*}; d=${cd#*:}
  timeout -k 10 500 python scripts/dev/ab_libs.py $c $d 4 build/var/lib_short.so build/var/lib_map3200.so > $O/map_${c}_$d.txt 2>&1 || { tail -5 $O/map_${c}_$d.txt; exit 1; }
  grep median $O/map_${c}_$d.txt | grep -v instance
done
