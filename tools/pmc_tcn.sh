# Three PMC passes (SQ counters, 8 per pass) of a short bench run; per-dispatch averages per kernel.
# usage (GPU box): bash tools/pmc_tcn.sh <tag>
set -o pipefail
tag=${1:-pmc}
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
run="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
B="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH SQ_LDS_ADDR_CONFLICT"
timeout -s KILL 90 rocprofv3 --pmc $A --output-format csv -d $out/a -o run -- $run > $out/a.log 2>&1 \
&& timeout -s KILL 90 rocprofv3 --pmc $B --output-format csv -d $out/b -o run -- $run > $out/b.log 2>&1 \
&& timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $out/c -o run -- $run > $out/c.log 2>&1 \
&& python3 tools/pmc_summary.py $out/a $out/b $out/c > $out/summary.txt && cat $out/summary.txt
