# k_tcn16 phase probe + launch shape + determinism (GPU box). usage: bash tools/r04_probe.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04p}; out=gpurun_out/$tag; mkdir -p $out
SEPVAD_TCN_INFO=1 timeout -k 10 200 python tools/det16.py > $out/det.log 2>&1; rc=$?; tail -30 $out/det.log; [ $rc -eq 0 ] || exit $rc
for t in 1 0; do
  SEPVAD_TCN16=$t SEPVAD_TCN_PROBE=$PWD/$out/probe_t$t.bin SEPVAD_TCN_INFO=1 timeout -k 10 120 python3 bench.py --steps 2 --warmup 2 \
      --no-cpu-baseline > $out/bench_probe_t$t.json 2> $out/bench_probe_t$t.err || exit 1
  grep sepvad: $out/bench_probe_t$t.err | tail -1
  python3 tools/tcn_probe.py $out/probe_t$t.bin > $out/phases_t$t.txt || exit 1
  echo "== k_tcn16=$t"; cat $out/phases_t$t.txt
done
python3 tools/tcn_probe.py $out/probe_t1.bin pairs
