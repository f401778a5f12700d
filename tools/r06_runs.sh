# Round 6: XCD runs for long groups (tcn_kernel.h RUN). Long-file tests, then interleaved lines with SEPVAD_TCN_RUNS=1/0
# at 30 s, 60 s and 125 s files, and the 60 s phase probe with runs. usage: bash tools/r06_runs.sh <tag> [rounds]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r06r}; R=${2:-3}; out=gpurun_out/$tag; mkdir -p $out
step() { echo "== $1 $(date +%T)"; }
step tests && timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_boundary.py -m gpu -x -v --timeout 300 --timeout-method thread \
   -k "whole_file or long or concurrent_long" > $out/pytest.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/pytest.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit $rc; }
step lines
for r in $(seq $R); do for runs in 1 0; do for w in "30:--samples 480000 --batch 4" "60:--samples 960000 --batch 2" "125:--samples 2000000 --batch 1"; do
  n=${w%%:*}; a=${w#*:}
  SEPVAD_TCN_RUNS=$runs timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload long $a > $out/l.json 2> $out/l.err || { tail -3 $out/l.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); print('long$n runs=$runs', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done; done; done | tee $out/lines.txt
step probe60 && SEPVAD_TCN_PROBE=$PWD/$out/p.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 20 --no-cpu-baseline --workload long --samples 960000 --batch 2 > $out/p.json 2> $out/p.err \
&& python3 tools/tcn_probe.py $out/p.bin > $out/phases_long60_runs.txt && rm -f $out/p.bin && head -22 $out/phases_long60_runs.txt
