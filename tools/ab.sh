# A/B timing of library variants on one GPU box: bench.py alternately with each .so, R rounds.
# usage: bash tools/ab.sh <tag> <rounds> libA.so libB.so [...]   (prints value and the k_tcn launch time)
set -o pipefail
tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for r in $(seq 1 $rounds); do
  for lib in "$@"; do
    n=$(basename $lib .so)
    SEPVAD_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --no-cpu-baseline > $out/$n.$r.json 2> $out/$n.$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('$out/$n.$r.json').read().strip().splitlines()[-1]); print('$n', $r, d['value'], d['roofline']['avg_launch_us'], d['ms_per_step'])"
  done
done
