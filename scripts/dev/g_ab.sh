# usage: scripts/dev/g_ab.sh OUT ROUNDS "cfg:dir[:packets] ..." lib1 lib2 ...   (GPU box; in-process A/B per config)
export TMPDIR=/tmp; O=gpurun_out/$1; R=$2; C=$3; shift 3; mkdir -p $O
for cd in $C; do
  IFS=: read c d np <<< "$cd"
  AB_PACKETS=${np:-0} timeout -k 10 400 python scripts/dev/ab_libs.py $c $d $R "$@" > $O/${c}_${d}_${np:-def}.txt 2>&1 || { tail -5 $O/${c}_${d}_${np:-def}.txt; exit 1; }
  echo "== $cd"; grep -v instance $O/${c}_${d}_${np:-def}.txt | grep median | sed 's/  all \[.*//'
done
