# Fused exact-fp32 arm: its parity / schedule tests, then the fp32 bench line next to the multi-kernel schedule's.
# usage: bash tools/r05_fp32.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05f}; mkdir -p $out
export SEPVAD_VAD_LABEL_LOG=$out/vad_labels.txt
step() { echo "== $1 $(date +%T)"; }
step pytest && timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "fp32 or two_slices" > $out/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $out/pytest.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit $rc; }
step bench_fp32 && timeout -k 10 300 python3 bench.py --no-cpu-baseline --precision fp32 > $out/fp32.json 2> $out/fp32.err \
&& step bench_fp32_mk && SEPVAD_FUSED=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline --precision fp32 > $out/fp32_mk.json 2> $out/fp32_mk.err \
&& for f in fp32 fp32_mk; do python3 -c "import json; d=json.loads(open('$out/$f.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], d['schedule'], r['avg_launch_us'], r['frac'])"; done
