# Round-4 roofline evidence for profiles/ (run on the GPU box from the repo root): rocprofv3 kernel stats of the
# headline command, HBM bytes (FETCH_SIZE x2 + WRITE_SIZE), texture-path counters, SQ counters, L2 hit rate, the
# MFMA/VALU co-issue counter, and (where the counter exists) the L2's DRAM-side read requests.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04prof
mkdir -p $out
bench="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline"
short="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
K="k_tcn<2, 1, false, 2, false, false>"
step() { echo "== $1 $(date +%T)"; }
step avail && { timeout -k 10 120 rocprofv3 --list-avail > $out/avail.txt 2>&1 || true; } \
&& step stats && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- $bench > $out/prof.log 2>&1 \
&& python3 tools/kstats.py $(find $out/prof -name "*kernel_stats.csv" | head -1) \
&& step fetch && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- $short > $out/pmc_fetch.log 2>&1 \
&& step write && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run -- $short > $out/pmc_write.log 2>&1 \
&& python3 tools/pmc.py $out/pmc_fetch $out/pmc_write "$K" $out/pmc_tcn.json \
&& step ta && bash tools/pmc_ta.sh r04prof/ta \
&& step sq && bash tools/pmc_tcn.sh r04prof/sq > /dev/null \
&& step tcc && timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/tcc -o run -- $short > $out/tcc.log 2>&1 \
&& python3 tools/pmc_summary.py $out/tcc > $out/tcc_summary.txt || exit 1
step coexec
if grep -q "SQ_VALU_MFMA_COEXEC_CYCLES" $out/avail.txt; then
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $out/coexec -o run -- $short > $out/coexec.log 2>&1 \
  && python3 tools/pmc_summary.py $out/coexec > $out/coexec_summary.txt || exit 1
else echo "SQ_VALU_MFMA_COEXEC_CYCLES not in rocprofv3 --list-avail" > $out/coexec_summary.txt; fi
step dram
if grep -q "TCC_EA0_RDREQ_DRAM" $out/avail.txt; then
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum --output-format csv -d $out/dram -o run -- $short > $out/dram.log 2>&1 \
  && python3 tools/pmc_summary.py $out/dram > $out/dram_summary.txt || exit 1
else echo "TCC_EA0_RDREQ_DRAM not in rocprofv3 --list-avail" > $out/dram_summary.txt; fi
step done
