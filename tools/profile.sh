# rocprofv3 kernel trace + stats of the default bench workload (B=64, N=32000, config_with_vad).
# usage (on the GPU box): bash tools/profile.sh <tag>
set -o pipefail
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/prof_$tag
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$tag/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
find gpurun_out/prof_$tag -name "*stats*" | head
exit $rc
