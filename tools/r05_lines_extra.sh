# The remaining round-5 lines at the steady-state window: exact fp32 fused / multi-kernel, one-slice cfg 3 / 4 / 5.
# usage: bash tools/r05_lines_extra.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r05lx}; mkdir -p $out
run() { n=$1; shift; echo "== $n $(date +%T)"; timeout -k 10 300 python3 bench.py "$@" > $out/$n.json 2> $out/$n.err && tail -1 $out/$n.json | cut -c1-120; }
run cfg2_fp32_fused --no-cpu-baseline --precision fp32 \
&& SEPVAD_FUSED=0 run cfg2_fp32_multikernel --no-cpu-baseline --precision fp32 \
&& SEPVAD_TCN_SLICES=1 run cfg3_stream_s1 --no-cpu-baseline --workload stream \
&& SEPVAD_TCN_SLICES=1 run cfg4_s1 --no-cpu-baseline --workload cfg4 \
&& SEPVAD_TCN_SLICES=1 run cfg5_s1 --no-cpu-baseline --workload cfg5
