# A/B of whole-forward bench lines (ms_per_step) between library variants, alternating, same box.
# usage: bash tools/ab_bench.sh <tag> <rounds> <bench args> -- libA.so[@VAR=value] libB.so ...
set -o pipefail
tag=$1; rounds=$2; shift 2
args=(); while [ "$1" != "--" ]; do args+=("$1"); shift; done; shift
out=gpurun_out/$tag; mkdir -p $out
for r in $(seq 1 $rounds); do
  for spec in "$@"; do
    lib=${spec%%@*}; envs=""; n=$(basename $lib .so)
    if [ "$spec" != "$lib" ]; then envs=${spec#*@}; n=$n.${envs##*=}; fi
    env $envs SEPVAD_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline "${args[@]}" > $out/$n.$r.json 2> $out/$n.$r.err || exit 1
    echo "$n $r $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'value', d['value'])" $out/$n.$r.json)"
  done
done | tee $out/abb.txt
python3 - $out/abb.txt <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    f = l.split(); d[f[0]].append(float(f[3]))
for n, xs in d.items():
    print(f"median {n:24s} ms_per_step {statistics.median(xs):.4f}  ({len(xs)} runs)")
PY
