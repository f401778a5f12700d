# One GPU call: library A/B in k_tcn shader cycles, then the whole GPU suite on the default library.
# usage: bash tools/step_ab_tests.sh <tag> <rounds> <launches> libA.so libB.so ...
set -o pipefail
tag=$1; rounds=$2; R=$3; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out/$tag
bash tools/ab_cyc.sh ${tag}_ab $rounds $R "$@" || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1
rc=$?
tail -8 gpurun_out/$tag/pytest.log
exit $rc
