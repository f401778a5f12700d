# Interleaved bench lines (cfg 2 and cfg 5, bench's steady window) of abl/lib_<name>.so variants.
# usage: bash tools/r06_lines4.sh <tag> <rounds> name1 name2 ...
set -o pipefail
export TMPDIR=/tmp
tag=$1; R=$2; shift 2; out=gpurun_out/$tag; mkdir -p $out
for r in $(seq $R); do for w in offline cfg5; do for n in "$@"; do
  SEPVAD_LIB=$PWD/abl/lib_$n.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload $w > $out/l.json 2> $out/l.err || { tail -3 $out/l.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); print('$w $n', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done; done; done | tee $out/lines.txt
python3 - $out/lines.txt <<'PY'
import sys, statistics, collections
v = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    w, n, val, ms, us = ln.split(); v[(w, n)].append((float(val), float(us)))
for k, xs in sorted(v.items()): print(k[0], k[1], 'median', statistics.median(x[0] for x in xs), 'k_tcn', statistics.median(x[1] for x in xs), 'n', len(xs))
PY
