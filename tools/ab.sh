# A/B timing of library variants on one GPU box: bench.py alternately with each .so, R rounds.
# usage: [AB_ARGS="--precision bf16"] bash tools/ab.sh <tag> <rounds> libA.so libB.so[@VAR=value] [...]
#   (lib@VAR=value: that run with the environment variable set, e.g. var/lib_x.so@SEPVAD_TCN_IMPL=1)
# prints per run: variant, round, utt/s, k_tcn average launch (us), ms per step; then medians per variant
set -o pipefail
tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for r in $(seq 1 $rounds); do
  for spec in "$@"; do
    lib=${spec%%@*}; envs=""; n=$(basename $lib .so)
    if [ "$spec" != "$lib" ]; then envs=${spec#*@}; n=$n.${envs##*=}; fi
    env $envs SEPVAD_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --no-cpu-baseline $AB_ARGS > $out/$n.$r.json 2> $out/$n.$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$out/$n.$r.json').read().strip().splitlines()[-1]); print('$n', $r, d['value'], d['roofline']['avg_launch_us'], d['ms_per_step'])"
  done
done | tee $out/ab.txt
python3 - $out/ab.txt <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    n, r, v, us, ms = l.split()
    d[n].append((float(v), float(us)))
for n, xs in d.items():
    print(f"median {n:12s} utt/s {statistics.median(x[0] for x in xs):9.1f}  k_tcn {statistics.median(x[1] for x in xs):7.1f} us")
PY
