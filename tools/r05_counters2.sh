# SQ / TA / co-issue / L2 / HBM counters of the two-slice k_tcn (cfg 5) and the long-group k_tcn (60 s files), each pass
# in a run of its own. usage: bash tools/r05_counters2.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05c}; mkdir -p $out
step() { echo "== $1 $(date +%T)"; }
for w in "cfg5" "long --samples 960000 --batch 2"; do
  n=${w%% *}
  run="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --workload $w"
  A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
  B="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
  C="SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA"
  D="TA_BUSY_avr TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE"
  step "$n sq" \
  && timeout -s KILL 120 rocprofv3 --pmc $A --output-format csv -d $out/$n/a -o run -- $run > $out/$n.a.log 2>&1 \
  && timeout -s KILL 120 rocprofv3 --pmc $B --output-format csv -d $out/$n/b -o run -- $run > $out/$n.b.log 2>&1 \
  && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $out/$n/c -o run -- $run > $out/$n.c.log 2>&1 \
  && timeout -s KILL 120 rocprofv3 --pmc $D --output-format csv -d $out/$n/d -o run -- $run > $out/$n.d.log 2>&1 \
  && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/$n/f -o run -- $run > $out/$n.f.log 2>&1 \
  && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/$n/w -o run -- $run > $out/$n.w.log 2>&1 \
  && python3 tools/pmc_summary.py $out/$n/a $out/$n/b $out/$n/c $out/$n/d > $out/${n}_summary.txt \
  && grep -A1 "k_tcn" $out/${n}_summary.txt \
  && python3 tools/pmc.py $out/$n/f $out/$n/w "k_tcn" $out/${n}_pmc_tcn.json || exit 1
done
step done
