# Weight lo-plane format at one and two slices: cfg 2 (one slice) and cfg 5 (two slices) with --wlo f16 / i8, alternating.
# usage: bash tools/r05_wlo.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r05w}; mkdir -p $out
for r in 1 2; do
  for wl in i8 f16; do
    for w in offline cfg5; do
      timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload $w --wlo $wl > $out/l.json 2> /dev/null || exit 1
      python3 -c "import json; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$w $wl $r', d['value'], d['ms_per_step'], r.get('avg_launch_us'))"
    done
  done
done | tee $out/wlo.txt
