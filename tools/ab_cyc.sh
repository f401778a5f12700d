# A/B of library variants in k_tcn SHADER CYCLES (launch span x workgroup 0's shader clock, tools/jitter.py): the
# launch-to-launch spread in time is the shader clock (corr 0.98, profiles/r03l_jitter.txt), in cycles it is 0.5 %.
# usage: bash tools/ab_cyc.sh <tag> <rounds> <launches> libA.so libB.so[@VAR=value] ...
set -o pipefail
tag=$1; rounds=$2; R=$3; shift 3
out=gpurun_out/$tag; mkdir -p $out
for r in $(seq 1 $rounds); do
  for spec in "$@"; do
    lib=${spec%%@*}; envs=""; n=$(basename $lib .so)
    if [ "$spec" != "$lib" ]; then envs=${spec#*@}; n=$n.${envs##*=}; fi
    env $envs SEPVAD_TCN_CLOCK=1 SEPVAD_LIB=$PWD/$lib timeout -k 10 120 python3 tools/jitter.py $R > $out/$n.$r.txt 2>&1 || exit 1
    echo "$n $r $(grep '^SUMMARY' $out/$n.$r.txt)"
  done
done | tee $out/abc.txt
python3 - $out/abc.txt <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    f = l.split()
    d[f[0]].append((float(f[4]), float(f[6]), float(f[8])))
for n, xs in d.items():
    print(f"median {n:14s} k_tcn {statistics.median(x[0] for x in xs):7.1f} us  {statistics.median(x[1] for x in xs):.4f} Mcycles"
          f"  ({statistics.median(x[2] for x in xs):.0f} MHz)")
PY
