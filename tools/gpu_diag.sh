# Diagnostics pass (GPU box): per-workgroup GEMM timeline probe and SQ/TCC counters of the TCN kernels.
set -o pipefail
out=gpurun_out/${1:-diag}
mkdir -p $out
export TMPDIR=/tmp
b="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 120 python3 tools/probe.py --block 5 > $out/probe.log 2>&1 && cat $out/probe.log \
&& timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS --output-format csv -d $out/sq -o run -- $b > $out/sq.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/tcc -o run -- $b > $out/tcc.log 2>&1 \
&& python3 tools/pmc_summary.py $out/sq $out/tcc
