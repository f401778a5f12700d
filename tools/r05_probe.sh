# Phase probes of k_tcn (one-slice at cfg 2, two-slice at cfg 5) and the cfg 3 streaming line with both widths.
# usage: bash tools/r05_probe.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05p}; mkdir -p $out
step() { echo "== $1 $(date +%T)"; }
step probe_cfg2 && SEPVAD_TCN_PROBE=$PWD/$out/probe_cfg2.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline > $out/p2.json 2> $out/p2.err \
&& python3 tools/tcn_probe.py $out/probe_cfg2.bin > $out/phases_cfg2.txt && head -16 $out/phases_cfg2.txt \
&& step probe_cfg5 && SEPVAD_TCN_PROBE=$PWD/$out/probe_cfg5.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --workload cfg5 > $out/p5.json 2> $out/p5.err \
&& python3 tools/tcn_probe.py $out/probe_cfg5.bin > $out/phases_cfg5.txt && head -16 $out/phases_cfg5.txt \
&& step stream2 && timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload stream > $out/stream.json 2> $out/stream.err && tail -1 $out/stream.json | cut -c1-200 \
&& step stream1 && SEPVAD_TCN_SLICES=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload stream > $out/stream_s1.json 2> $out/stream_s1.err && tail -1 $out/stream_s1.json | cut -c1-200 \
&& step long60 && timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload long --samples 960000 --batch 2 > $out/long60.json 2> $out/long60.err && tail -1 $out/long60.json | cut -c1-200
