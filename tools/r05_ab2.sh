# k_stft_gate at 16 own frames (3 per CU) and static wave priority, against var/lib_pit.so: parity suite, digests,
# alternating cfg 2 / cfg 5 / cfg 3 lines with kernel stats. usage: bash tools/r05_ab2.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05q}; mkdir -p $out
export SEPVAD_VAD_LABEL_LOG=$out/vad_labels.txt
step() { echo "== $1 $(date +%T)"; }
step pytest && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $out/pytest.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit $rc; }
step digests
for bn in "64 32000" "128 32000" "2 960000"; do
  for lib in var/lib_pit.so var/lib_stft.so var/lib_prio.so; do SEPVAD_LIB=$PWD/$lib timeout -k 10 120 python3 tools/bitwise_ab.py $bn 2>/dev/null | tail -1 || exit 1; done
done | tee $out/digests.txt
step lines
for r in 1 2; do
  for lib in var/lib_pit.so var/lib_stft.so var/lib_prio.so; do
    n=$(basename $lib .so)
    for w in offline cfg5 stream; do
      SEPVAD_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $w > $out/l.json 2> /dev/null || exit 1
      python3 -c "import json,sys; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$n', sys.argv[1], $r, d['value'], d['ms_per_step'], r.get('avg_launch_us'))" $w
    done
  done
done | tee $out/lines.txt
for lib in var/lib_pit.so var/lib_stft.so; do
  n=$(basename $lib .so)
  SEPVAD_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$n -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --workload cfg5 > /dev/null 2>&1 || exit 1
  echo "$n cfg5"; python3 tools/kstats.py $(find $out/prof_$n -name "*kernel_stats.csv" | head -1) | grep -E "stft|istft|k_tcn"
done | tee $out/stats.txt
step done
