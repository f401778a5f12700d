# Kernel stats of the cfg 3 streaming line and the 60 s file line (where their time goes).
# usage: bash tools/r05_wprof.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05w}; mkdir -p $out
step() { echo "== $1 $(date +%T)"; }
step stream && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stream -o run -- python3 bench.py --no-cpu-baseline --workload stream --steps 3 --warmup 1 > $out/stream.json 2> $out/stream.err \
&& python3 tools/kstats.py $(find $out/stream -name "*kernel_stats.csv" | head -1) \
&& step long60 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/long60 -o run -- python3 bench.py --no-cpu-baseline --workload long --samples 960000 --batch 2 --steps 10 --warmup 2 > $out/long60.json 2> $out/long60.err \
&& python3 tools/kstats.py $(find $out/long60 -name "*kernel_stats.csv" | head -1) \
&& step done
