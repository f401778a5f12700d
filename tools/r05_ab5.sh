# Bitwise digests and k_tcn shader cycles (cfg 2) of two libraries, then cfg 5 lines. usage: bash tools/r05_ab5.sh <tag> libA libB
set -o pipefail
export TMPDIR=/tmp
tag=$1; A=$2; B=$3; out=gpurun_out/$tag; mkdir -p $out
for bn in "64 32000" "128 32000"; do
  for lib in $A $B; do SEPVAD_LIB=$PWD/$lib timeout -k 10 120 python3 tools/bitwise_ab.py $bn 2>/dev/null | tail -1 || exit 1; done
done | tee $out/digests.txt
bash tools/ab_cyc.sh $tag/cyc 5 30 $A $B | tail -2 || exit 1
for r in 1 2; do for lib in $A $B; do
  SEPVAD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload cfg5 > $out/l.json 2> /dev/null || exit 1
  python3 -c "import json; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$(basename $lib) cfg5 $r', d['value'], r.get('avg_launch_us'))"
done; done | tee $out/lines.txt
