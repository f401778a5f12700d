# Precision arms on the GPU box: the tolerance sweep, all GPU tests, one bench line per arm.
# usage: bash tools/prec_round.sh <tag>
set -o pipefail
tag=${1:-prec}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py -x -v -s --timeout 300 --timeout-method thread \
    > $out/precision.log 2>&1; rc=$?; grep '^{' $out/precision.log; [ $rc -eq 0 ] || { tail -30 $out/precision.log; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 \
    || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for p in f16x3 bf16 f16; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --precision $p > $out/bench_$p.json 2> $out/bench_$p.err || exit 1
  python3 -c "import json; d=json.loads(open('$out/bench_$p.json').read().strip().splitlines()[-1]); print('$p', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
