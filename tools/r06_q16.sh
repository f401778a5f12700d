# Round 6: ring depth 8 vs 16 (int8 lo plane) in wall time: steady-state cfg 2 lines and the driver's 20 + 5 command,
# interleaved. usage: bash tools/r06_q16.sh <tag> <rounds> name1 name2
set -o pipefail
export TMPDIR=/tmp
tag=$1; R=$2; shift 2; out=gpurun_out/$tag; mkdir -p $out
for r in $(seq $R); do for mode in steady driver; do for n in "$@"; do
  if [ $mode = steady ]; then args=""; else args="--steps 20 --warmup 5"; fi
  SEPVAD_LIB=$PWD/abl/lib_$n.so timeout -k 10 200 python3 bench.py --no-cpu-baseline $args > $out/l.json 2> $out/l.err || { tail -3 $out/l.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); print('$mode $n', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done; done; done | tee $out/lines.txt
python3 - $out/lines.txt <<'PY'
import sys, statistics, collections
v = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    w, n, val, ms, us = ln.split(); v[(w, n)].append((float(val), float(us)))
for k, xs in sorted(v.items()): print(k[0], k[1], 'median', statistics.median(x[0] for x in xs), 'k_tcn', statistics.median(x[1] for x in xs), 'n', len(xs))
PY
