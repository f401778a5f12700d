# PIT sums / choose parallelised: streaming tests, the remainder-groups test, cfg 3 line A/B against the previous library,
# kernel stats of cfg 3. usage: bash tools/r05_pit.sh <tag> <previous lib>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05t}; prev=$2; mkdir -p $out
export SEPVAD_VAD_LABEL_LOG=$out/vad_labels.txt
step() { echo "== $1 $(date +%T)"; }
step pytest && timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_fused.py -m gpu -x -v --timeout 240 --timeout-method thread -k "stream or pit or remainder or online" > $out/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $out/pytest.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit $rc; }
for r in 1 2; do
  for lib in $prev sep-tfanet-vad_amd/libsepvad.so; do
    SEPVAD_LIB=$PWD/$lib SEPVAD_BENCH_DUMP=$PWD/$out/dump_$(basename $lib .so) timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload stream > $out/s.json 2> /dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$out/s.json').read().strip().splitlines()[-1]); print('$(basename $lib) $r', d['value'], d['ms_per_step'])"
  done
done | tee $out/ab.txt
python3 - $out $(basename $prev .so) <<'PY' | tee -a $out/ab.txt
import glob, sys
import numpy as np
out, prev = sys.argv[1], sys.argv[2]
a = np.load(glob.glob(f"{out}/dump_{prev}*.npy")[0]); b = np.load(glob.glob(f"{out}/dump_libsepvad*.npy")[0])
print("stitched streams bitwise equal:", np.array_equal(a.view(np.uint32), b.view(np.uint32)))
PY
step stats && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --no-cpu-baseline --workload stream --steps 3 --warmup 1 > $out/prof.log 2>&1 \
&& python3 tools/kstats.py $(find $out/prof -name "*kernel_stats.csv" | head -1) | grep -v copyBuffer
step done
rm -f $out/dump_*.npy  # (tens of MB: keep gpurun_out under the copy-back limit)
