# Interleaved bench lines of two libraries (same box), N rounds. usage: bash tools/r05_ab_lines.sh <tag> libA libB rounds [bench args]
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; A=$2; B=$3; R=$4; shift 4; mkdir -p $out
for r in $(seq $R); do for lib in $A $B; do
  SEPVAD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > $out/l.json 2> /dev/null || exit 1
  python3 -c "import json; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); print('$(basename $lib .so)', d['value'], d['ms_per_step'])"
done; done | tee $out/lines.txt
python3 - $out/lines.txt <<'PY'
import sys, statistics, collections
v = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    k, val, ms = ln.split(); v[k].append(float(val))
for k, xs in v.items(): print(k, 'median', statistics.median(xs), 'mean', round(statistics.mean(xs), 1), 'n', len(xs))
PY
