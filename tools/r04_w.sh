# k_tcn16 4 vs 8 waves: determinism / parity vs k_tcn (B=64) and the phase probe. usage: bash tools/r04_w.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04w}; out=gpurun_out/$tag; mkdir -p $out
for w in 8 4; do
  SEPVAD_TCN16_WAVES=$w SEPVAD_TCN_INFO=1 timeout -k 10 200 python tools/det16.py 64 32000 > $out/det_w$w.log 2>&1 || { tail -5 $out/det_w$w.log; exit 1; }
  echo "== waves $w"; grep -E "run . sep|k_tcn16 vs k_tcn sep|k_tcn16 grid" $out/det_w$w.log | sort | uniq -c
  SEPVAD_TCN16=1 SEPVAD_TCN16_WAVES=$w SEPVAD_TCN_PROBE=$PWD/$out/probe_w$w.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 2 \
      --no-cpu-baseline > $out/bench_probe_w$w.json 2> $out/bench_probe_w$w.err || exit 1
  python3 tools/tcn_probe.py $out/probe_w$w.bin > $out/phases_w$w.txt || exit 1
  head -16 $out/phases_w$w.txt
  SEPVAD_TCN16=1 SEPVAD_TCN16_WAVES=$w timeout -k 10 120 python3 bench.py --no-cpu-baseline > $out/bench_w$w.json 2> $out/bench_w$w.err || exit 1
  tail -1 $out/bench_w$w.json | cut -c1-200
done
