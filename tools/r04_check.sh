# k_tcn16 bring-up on the GPU box: parity tests, then bench with k_tcn16 on / off. usage: bash tools/r04_check.sh <tag> [tests]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04}; tests=${2:-tests/test_gpu_parity.py}
out=gpurun_out/$tag; mkdir -p $out
SEPVAD_TCN16=${T16:-1} timeout -k 10 600 python -u -m pytest $tests -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
tail -5 $out/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for t in 1 0; do
  SEPVAD_TCN16=$t timeout -k 10 200 python3 bench.py --no-cpu-baseline > $out/bench_t$t.json 2> $out/bench_t$t.err || exit $?
  tail -1 $out/bench_t$t.json | cut -c1-420
done
exit $rc
