# A/B of two library builds: bitwise digests (cfg 2, cfg 5, 60 s), k_tcn shader cycles at cfg 2 (tools/ab_cyc.sh), and
# alternating bench lines (cfg 2, cfg 5, 60 s) with the k_tcn launch time. usage: bash tools/r05_ab.sh <tag> libA libB
set -o pipefail
export TMPDIR=/tmp
tag=$1; A=$2; B=$3
out=gpurun_out/$tag; mkdir -p $out
step() { echo "== $1 $(date +%T)"; }
step digests
for bn in "64 32000" "128 32000" "2 960000"; do
  for lib in $A $B; do SEPVAD_LIB=$PWD/$lib timeout -k 10 120 python3 tools/bitwise_ab.py $bn 2>/dev/null | tail -1 || exit 1; done
done | tee $out/digests.txt
step cycles && bash tools/ab_cyc.sh $tag/cyc 4 30 $A $B | tail -2 || exit 1
step lines
for r in 1 2; do
  for lib in $A $B; do
    n=$(basename $lib .so)
    for w in "offline" "cfg5" "long --samples 960000 --batch 2"; do
      SEPVAD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload $w > $out/l.json 2> /dev/null || exit 1
      python3 -c "import json,sys; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$n', sys.argv[1], $r, d['value'], d['ms_per_step'], r.get('avg_launch_us'))" ${w%% *}
    done
  done
done | tee $out/lines.txt
step done
