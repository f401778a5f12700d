set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_configs.py tests/test_gpu_stream.py > gpurun_out/r04db_tests.log 2>&1 || { grep -E "passed|failed|Error|assert" gpurun_out/r04db_tests.log | head -20; exit 1; }
tail -1 gpurun_out/r04db_tests.log
mkdir -p gpurun_out/r04dbp
SEPVAD_TAIL_PROBE=$PWD/gpurun_out/r04dbp/t timeout -k 10 200 python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline > gpurun_out/r04dbp/b.json 2>&1 || exit 1
python3 tools/tail_probe.py gpurun_out/r04dbp/t.stft
timeout -k 10 800 bash tools/ab_bench.sh r04db_bench 5 --steps 200 --warmup 20 -- sep-tfanet-vad_amd/libsepvad_dbslow.so sep-tfanet-vad_amd/libsepvad.so
