# Phase probe of k_tcn on long files (16 s, 60 s) and cfg 2. usage: bash tools/probe_long.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-plong}; mkdir -p $out
run() { n=$1; shift
  SEPVAD_TCN_PROBE=$PWD/$out/probe_$n.bin timeout -k 10 180 python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline "$@" \
      > $out/bench_probe_$n.json 2> $out/bench_probe_$n.err || return 1
  python3 tools/tcn_probe.py $out/probe_$n.bin > $out/phases_$n.txt || return 1
  echo "== $n"; head -17 $out/phases_$n.txt; }
run long60 --workload long --samples 960000 --batch 2 && run long16 --workload long && run cfg2
