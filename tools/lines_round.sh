# Every bench line of DESIGN.md §7 on one GPU box: offline fp16x3 (with CPU baseline) and bf16, cfg4,
# cfg5 x {fp16x3, f16, bf16}, cfg3 streaming, 16 s and 30 s files (fused and multi-kernel), 60 s files, the opt-in
# weight lo planes. usage: bash tools/lines_round.sh <tag>
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
&& SEPVAD_FUSED=0 run long_multikernel --no-cpu-baseline --workload long \
&& run long30_f16x3 --no-cpu-baseline --workload long --samples 480000 --batch 4 \
&& SEPVAD_FUSED=0 run long30_multikernel --no-cpu-baseline --workload long --samples 480000 --batch 4 \
&& run long60_f16x3 --no-cpu-baseline --workload long --samples 960000 --batch 2 \
&& run offline_wlo_i8 --no-cpu-baseline --wlo i8 \
&& run offline_wlo_e4m3 --no-cpu-baseline --wlo e4m3 \
&& run long125_f16x3 --no-cpu-baseline --workload long --samples 2000000 --batch 1 \
&& run long125_b2_f16x3 --no-cpu-baseline --workload long --samples 2000000 --batch 2
