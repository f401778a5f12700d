# Focused A/B: k_tcn shader cycles at cfg 2 (pit vs prio, interleaved), kernel stats at cfg 2 (pit, stft, prio).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05r}; mkdir -p $out
bash tools/ab_cyc.sh ${1:-r05r}/cyc 5 30 var/lib_pit.so var/lib_prio.so var/lib_stft.so | tail -3 || exit 1
for lib in var/lib_pit.so var/lib_stft.so var/lib_prio.so; do
  n=$(basename $lib .so)
  SEPVAD_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$n -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  echo "$n cfg2"; python3 tools/kstats.py $(find $out/prof_$n -name "*kernel_stats.csv" | head -1) | grep -E "stft|istft|k_tcn|vad_feat"
done | tee $out/stats.txt
