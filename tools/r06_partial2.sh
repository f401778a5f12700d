# cfg 2 at T = 126 and T = 128, cfg 5 and cfg 3 (streaming) lines of two variants, interleaved. usage: bash tools/r06_partial2.sh <tag> A B
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; A=$2; B=$3; mkdir -p $out
for r in 1 2 3; do for n in $A $B; do for w in "offline --samples 32000" "offline --samples 32512" "cfg5" "cfg4"; do
  SEPVAD_LIB=$PWD/abl/lib_$n.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload $w > $out/l.json 2> $out/l.err || { tail -3 $out/l.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); print('$n', '$w'.replace(' ', '_'), d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done; done; done | tee $out/lines.txt
python3 - $out/lines.txt <<'PY'
import sys, statistics, collections
v = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    n, w, val, ms, us = ln.split(); v[(w, n)].append((float(val), float(us)))
for k, xs in sorted(v.items()): print(k[0], k[1], 'median', statistics.median(x[0] for x in xs), 'k_tcn', statistics.median(x[1] for x in xs))
PY
