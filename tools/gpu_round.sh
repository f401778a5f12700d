# Full GPU pass (run on the GPU box from the repo root): smoke, parity tests, bench, rocprofv3
# kernel stats and the two PMC passes for the dominant kernel's HBM traffic.
# usage: bash tools/gpu_round.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-r01}
skip=${2:-}
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
bench="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline"
step() { echo "== $1 $(date +%T)"; }

step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 \
&& tail -2 $out/smoke.log \
&& { [ -n "$skip" ] || { step pytest && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 \
       --timeout-method thread > $out/pytest.log 2>&1; rc=$?; tail -4 $out/pytest.log; [ $rc -eq 0 ]; }; } \
&& step bench && timeout -k 10 400 python3 bench.py > $out/bench.json 2> $out/bench.err \
&& cat $out/bench.json \
&& step rocprof && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run \
       -- $bench > $out/prof.log 2>&1 \
&& step pmc_fetch && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run \
       -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/pmc_fetch.log 2>&1 \
&& step pmc_write && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run \
       -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/pmc_write.log 2>&1 \
&& python3 tools/pmc.py $out/pmc_fetch $out/pmc_write "k_tcn<2, 1, false, 2, false>" $out/pmc_tcn.json \
&& python3 tools/kstats.py $(find $out/prof -name "*kernel_stats.csv" | head -1) \
&& step done
