set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_boundary.py tests/test_gpu_precision.py > gpurun_out/r04bd.log 2>&1; rc=$?
grep -E "passed|failed|round [0-9]|AssertionError" gpurun_out/r04bd.log | head -20; exit $rc
