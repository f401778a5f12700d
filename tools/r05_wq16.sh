# Two-slice k_tcn on the fp16 copy of the int8 lo plane: bitwise digests and interleaved lines. usage: bash tools/r05_wq16.sh <tag> libA libB
set -o pipefail
export TMPDIR=/tmp
tag=$1; A=$2; B=$3; out=gpurun_out/$tag; mkdir -p $out
for bn in "128 32000" "256 48000" "64 64000" "4 480000" "64 32000"; do
  for lib in $A $B; do SEPVAD_LIB=$PWD/$lib timeout -k 10 150 python3 tools/bitwise_ab.py $bn 2>/dev/null | tail -1 || exit 1; done
done | tee $out/digests.txt
for r in 1 2; do for w in cfg5 stream cfg4; do for lib in $A $B; do
  SEPVAD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload $w > $out/l.json 2> /dev/null || exit 1
  python3 -c "import json; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$(basename $lib) $w', d['value'], r.get('avg_launch_us'))"
done; done; done | tee $out/lines.txt
