set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_boundary.py > gpurun_out/r04x_tests.log 2>&1 || { tail -40 gpurun_out/r04x_tests.log; exit 1; }
tail -2 gpurun_out/r04x_tests.log
mkdir -p gpurun_out/r04xp
SEPVAD_TAIL_PROBE=$PWD/gpurun_out/r04xp/t timeout -k 10 200 python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline > gpurun_out/r04xp/b.json 2>&1 || exit 1
python3 tools/tail_probe.py gpurun_out/r04xp/t.istft && python3 tools/tail_probe.py gpurun_out/r04xp/t.stft
timeout -k 10 700 bash tools/ab_bench.sh r04x_bench 4 --steps 200 --warmup 20 -- sep-tfanet-vad_amd/libsepvad.so@SEPVAD_X_STORE=1 sep-tfanet-vad_amd/libsepvad.so
