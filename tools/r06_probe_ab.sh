# Round 6: k_tcn phase probes (cfg 2, after a 300-forward warm-up) of abl/lib_<name>.so variants.
# usage: bash tools/r06_probe_ab.sh <tag> name1 name2 ...
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out
for n in "$@"; do
  echo "== $n $(date +%T)"
  SEPVAD_LIB=$PWD/abl/lib_$n.so SEPVAD_TCN_PROBE=$PWD/$out/probe_$n.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 300 --no-cpu-baseline > $out/p_$n.json 2> $out/p_$n.err || { tail -3 $out/p_$n.err; exit 1; }
  python3 tools/tcn_probe.py $out/probe_$n.bin > $out/phases_$n.txt || exit 1
  rm -f $out/probe_$n.bin
  head -40 $out/phases_$n.txt
done
