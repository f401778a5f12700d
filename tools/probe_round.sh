# Phase probe of k_tcn on the GPU box: one forward with SEPVAD_TCN_PROBE, per precision arm.
# usage: bash tools/probe_round.sh <tag> [arms...]
set -o pipefail
tag=${1:-probe}; shift; arms=${@:-f16x3}
out=gpurun_out/$tag; mkdir -p $out
for p in $arms; do
  SEPVAD_TCN_PROBE=$PWD/$out/probe_$p.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline \
      --precision $p > $out/bench_probe_$p.json 2> $out/bench_probe_$p.err || exit 1
  python3 tools/tcn_probe.py $out/probe_$p.bin > $out/phases_$p.txt || exit 1
  echo "== $p"; cat $out/phases_$p.txt
done
