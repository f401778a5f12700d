# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of bench.py with each library variant.
# usage: bash tools/kstat_ab.sh <tag> libA.so libB.so ...
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so); out=gpurun_out/$tag/$n; mkdir -p $out
  SEPVAD_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run \
      -- python3 bench.py --steps ${KSTEPS:-10} --warmup 3 --no-cpu-baseline > $out/prof.log 2>&1 || exit 1
  echo "== $n"; python3 tools/kstats.py $(find $out -name "*kernel_stats.csv" | head -1) | grep sepvad || exit 1
done
