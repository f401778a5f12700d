# Texture-path (TA / TCP) counters of a short bench run: is k_tcn's weight stream bound by the per-CU
# vector-memory path? Three passes within the per-block limits (TA 2, TCP 4, GRBM 2).
# usage (GPU box): bash tools/pmc_ta.sh <tag>
set -o pipefail
tag=${1:-pmc_ta}
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
run="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
A="TA_BUSY_avr TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE"
B="TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
C="TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum"
timeout -s KILL 90 rocprofv3 --pmc $A --output-format csv -d $out/a -o run -- $run > $out/a.log 2>&1 \
&& timeout -s KILL 90 rocprofv3 --pmc $B --output-format csv -d $out/b -o run -- $run > $out/b.log 2>&1 \
&& timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $out/c -o run -- $run > $out/c.log 2>&1 \
&& python3 tools/pmc_summary.py $out/a $out/b $out/c > $out/summary.txt && grep -A1 k_tcn $out/summary.txt
