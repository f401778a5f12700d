# One GPU iteration: all GPU tests, the phase probe per arm, one bench line per arm.
# usage: bash tools/iter.sh <tag> [arms...]
set -o pipefail
tag=${1:-it}; shift; arms=${@:-f16x3 bf16}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 \
    || { grep -E "Error|assert|FAILED|Fatal" $out/pytest.log | head -30; tail -5 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
bash tools/probe_round.sh $tag $arms > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
grep -E "^==|per block|conv1d|epilogue|P1|dwconv|res_out|P2|rowsum|P3|gates|moments|P4|x' update" $out/probe.log | grep -v "per-wave\|    " 
for p in $arms; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --precision $p > $out/bench_$p.json 2> $out/bench_$p.err || exit 1
  python3 -c "import json; d=json.loads(open('$out/bench_$p.json').read().strip().splitlines()[-1]); print('$p', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
