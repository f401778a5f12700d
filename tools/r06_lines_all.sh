# Round 6: every bench line (tools/lines_round.sh) plus the exact-fp32 arms and the driver's own command (20 timed steps
# after 5 warmup steps) three times. usage: bash tools/r06_lines_all.sh <tag>
set -o pipefail
tag=${1:-r06_lines}; out=gpurun_out/$tag
bash tools/lines_round.sh $tag || exit 1
run() { n=$1; shift; echo "== $n $(date +%T)"; timeout -k 10 300 python3 bench.py "$@" > $out/$n.json 2> $out/$n.err && tail -1 $out/$n.json | cut -c1-160; }
run cfg2_fp32_fused --no-cpu-baseline --precision fp32 \
&& SEPVAD_FUSED=0 run cfg2_fp32_multikernel --no-cpu-baseline --precision fp32 \
&& run driver_20_5_a --steps 20 --warmup 5 \
&& run driver_20_5_b --steps 20 --warmup 5 --no-cpu-baseline \
&& run driver_20_5_c --steps 20 --warmup 5 --no-cpu-baseline
