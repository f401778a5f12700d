# The whole GPU suite + smoke + headline bench on the box. usage: bash tools/gpu_tests.sh <tag> [pytest args]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-gt}; shift
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread "$@" > $out/pytest.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/pytest.log | tail -3; grep -E "VAD labels" $out/pytest.log | sort | uniq -c | head -20
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head; exit $rc; }
timeout -k 10 300 python3 bench.py > $out/bench.json 2> $out/bench.err || exit 1
tail -1 $out/bench.json | cut -c1-300
