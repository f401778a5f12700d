# bench at each batch split (GPU box)
set -o pipefail
out=gpurun_out/${1:-split}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "split or strided or matches_reference" > $out/pytest.log 2>&1; rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for s in 1 2 3 4; do
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --split $s > $out/bench_s$s.json 2>$out/bench_s$s.err || exit $?
  python3 -c "import json,sys; d=json.load(open('$out/bench_s$s.json')); print('split', $s, d['value'], d['ms_per_step'])"
done
