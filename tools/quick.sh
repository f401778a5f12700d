# Quick GPU iteration: GPU parity tests, bench, kernel stats. usage: bash tools/quick.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-q}; skip=${2:-}
export TMPDIR=/tmp
out=gpurun_out/$tag; mkdir -p $out
{ [ -n "$skip" ] || { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/pytest.log 2>&1; rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ]; }; } \
&& timeout -k 10 300 python3 bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err && tail -1 $out/bench.json \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run \
    -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/prof.log 2>&1 \
&& python3 tools/kstats.py $(find $out/prof -name "*kernel_stats.csv" | head -1)
