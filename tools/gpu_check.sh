set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -le 1 ]; then timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest.log; fi
if [ $rc -le 1 ]; then timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 5 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log; fi
exit $rc
