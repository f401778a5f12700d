# Long-file fused path: fused tests, then the phase probe and bench lines for 16 / 30 / 60 s files. usage: bash tools/r04_long.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-rlong}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_boundary.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
tail -2 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit $rc; }
bash tools/probe_long.sh ${1:-rlong} | grep -E "==|per block|P3|P4|dwconv" || exit 1
run() { n=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > $out/$n.json 2> $out/$n.err && echo "$n $(tail -1 $out/$n.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["avg_launch_us"])')"; }
run long60 --workload long --samples 960000 --batch 2 && run long30 --workload long --samples 480000 --batch 4 && run long16 --workload long && run offline
