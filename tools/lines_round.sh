# Every bench line of DESIGN.md §7 on one GPU box: offline fp16x3 (with CPU baseline) and bf16, cfg4,
# cfg5 x {fp16x3, f16, bf16}, cfg3 streaming, 16 s files (fused and multi-kernel). usage: bash tools/lines_round.sh <tag>
set -o pipefail
out=gpurun_out/${1:-lines}; mkdir -p $out
run() { n=$1; shift; echo "== $n $(date +%T)"; timeout -k 10 300 python3 bench.py "$@" > $out/$n.json 2> $out/$n.err && tail -1 $out/$n.json | cut -c1-160; }
run offline_f16x3 \
&& run offline_bf16 --no-cpu-baseline --precision bf16 \
&& run cfg4_f16x3 --no-cpu-baseline --workload cfg4 \
&& run cfg5_f16x3 --no-cpu-baseline --workload cfg5 \
&& run cfg5_f16 --no-cpu-baseline --workload cfg5 --precision f16 \
&& run cfg5_bf16 --no-cpu-baseline --workload cfg5 --precision bf16 \
&& run stream_cfg3 --no-cpu-baseline --workload stream \
&& run long_f16x3 --no-cpu-baseline --workload long \
&& SEPVAD_FUSED=0 run long_multikernel --no-cpu-baseline --workload long
