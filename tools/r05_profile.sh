# Round-5 roofline evidence for profiles/ (GPU box, repo root), on the final tree: rocprofv3 kernel stats of the headline
# command (cfg 2, one-slice k_tcn) and of cfg 5 (two-slice k_tcn), HBM bytes (FETCH_SIZE x2 + WRITE_SIZE), texture-path
# and SQ counters, L2 hit rate, MFMA/VALU co-issue, DRAM-side read requests -- each counter pass in a run of its own.
# usage: bash tools/r05_profile.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r05prof}
out=gpurun_out/$tag
mkdir -p $out
bench="python3 bench.py --no-cpu-baseline"  # default steps: steady-state clocks (bench.py STEADY_STEPS)
short="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
K="k_tcn<2, 1, false, 2, false, false, 1>"
step() { echo "== $1 $(date +%T)"; }
step stats && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- $bench > $out/prof.log 2>&1 \
&& python3 tools/kstats.py $(find $out/prof -name "*kernel_stats.csv" | head -1) \
&& step stats_cfg5 && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof5 -o run -- $bench --workload cfg5 > $out/prof5.log 2>&1 \
&& python3 tools/kstats.py $(find $out/prof5 -name "*kernel_stats.csv" | head -1) \
&& step fetch && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- $short > $out/pmc_fetch.log 2>&1 \
&& step write && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run -- $short > $out/pmc_write.log 2>&1 \
&& python3 tools/pmc.py $out/pmc_fetch $out/pmc_write "$K" $out/pmc_tcn.json \
&& step ta && bash tools/pmc_ta.sh $tag/ta \
&& step sq && bash tools/pmc_tcn.sh $tag/sq > /dev/null \
&& step tcc && timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/tcc -o run -- $short > $out/tcc.log 2>&1 \
&& python3 tools/pmc_summary.py $out/tcc > $out/tcc_summary.txt \
&& step coexec && timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $out/coexec -o run -- $short > $out/coexec.log 2>&1 \
&& python3 tools/pmc_summary.py $out/coexec > $out/coexec_summary.txt \
&& step dram && timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum --output-format csv -d $out/dram -o run -- $short > $out/dram.log 2>&1 \
&& python3 tools/pmc_summary.py $out/dram > $out/dram_summary.txt \
&& step done
