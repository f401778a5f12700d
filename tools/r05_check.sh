# Round-5 check on the GPU box: the fused / parity suites (incl. the two-slice tests), then cfg 2 and cfg 5 bench lines
# with one- and two-slice workgroups. usage: bash tools/r05_check.sh <tag> [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r05}; kexpr=${2:-}
out=gpurun_out/$tag; mkdir -p $out
export SEPVAD_VAD_LABEL_LOG=$out/vad_labels.txt
step() { echo "== $1 $(date +%T)"; }
step pytest
if [ -n "$kexpr" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "$kexpr" > $out/pytest.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest.log 2>&1
fi
rc=$?; grep -E "passed|failed|error" $out/pytest.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit $rc; }
step bench_cfg2 && timeout -k 10 300 python3 bench.py --no-cpu-baseline > $out/cfg2.json 2> $out/cfg2.err \
&& step bench_cfg5_2 && timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload cfg5 > $out/cfg5.json 2> $out/cfg5.err \
&& step bench_cfg5_1 && SEPVAD_TCN_SLICES=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload cfg5 > $out/cfg5_s1.json 2> $out/cfg5_s1.err \
&& step bench_cfg4_2 && timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload cfg4 > $out/cfg4.json 2> $out/cfg4.err \
&& step bench_cfg4_1 && SEPVAD_TCN_SLICES=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload cfg4 > $out/cfg4_s1.json 2> $out/cfg4_s1.err \
&& for f in cfg2 cfg5 cfg5_s1 cfg4 cfg4_s1; do python3 -c "import json,sys; d=json.loads(open('$out/$f.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'])"; done
