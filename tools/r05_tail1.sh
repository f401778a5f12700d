# One-slice tail round after two-slice rounds: fused tests, cfg 3 line A/B (SEPVAD_TCN_TAIL1=0/1), a B = 100 T = 188
# batch with the launch shapes printed. usage: bash tools/r05_tail1.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05v}; mkdir -p $out
export SEPVAD_VAD_LABEL_LOG=$out/vad_labels.txt
step() { echo "== $1 $(date +%T)"; }
step pytest && timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $out/pytest.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit $rc; }
SEPVAD_TCN_INFO=1 timeout -k 10 120 python3 tools/bitwise_ab.py 100 48000 2>&1 | grep -E "k_tcn grid|libsepvad" | tee $out/shape.txt
SEPVAD_TCN_TAIL1=0 timeout -k 10 120 python3 tools/bitwise_ab.py 100 48000 2>&1 | grep libsepvad | tee -a $out/shape.txt
for r in 1 2 3; do
  for t in 0 1; do
    SEPVAD_TCN_TAIL1=$t timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload stream > $out/s.json 2> /dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$out/s.json').read().strip().splitlines()[-1]); print('tail1=$t round $r', d['value'], d['ms_per_step'])"
  done
done | tee $out/ab.txt
step done
