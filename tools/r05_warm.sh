# Headline line vs warmup / steps (clock ramp): usage: bash tools/r05_warm.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05warm}; mkdir -p $out
for r in 1 2; do for kw in "20 3" "20 100" "20 400" "200 20" "500 100" "2000 200"; do
  set -- $kw
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps $1 --warmup $2 > $out/l.json 2> /dev/null || exit 1
  python3 -c "import json; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); print('steps $1 warmup $2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done; done | tee $out/lines.txt
