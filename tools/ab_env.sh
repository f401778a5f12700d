# A/B timing of one library under two environment settings: bench.py alternately, R rounds.
# usage: bash tools/ab_env.sh <tag> <rounds> "VAR=a" "VAR=b"
set -o pipefail
tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for r in $(seq 1 $rounds); do
  for e in "$@"; do
    env $e timeout -k 10 120 python3 bench.py --no-cpu-baseline $AB_ARGS > $out/${e//=/_}.$r.json 2> $out/${e//=/_}.$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$out/${e//=/_}.$r.json').read().strip().splitlines()[-1]); print('${e//=/_}', $r, d['value'], d['roofline']['avg_launch_us'], d['ms_per_step'])"
  done
done | tee $out/ab.txt
python3 - $out/ab.txt <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    n, r, v, us, ms = l.split()
    d[n].append((float(v), float(ms)))
for n, xs in d.items():
    print(f"median {n:20s} utt/s {statistics.median(x[0] for x in xs):9.1f}  ms/step {statistics.median(x[1] for x in xs):7.4f}")
PY
