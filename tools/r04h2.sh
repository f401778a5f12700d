set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused.py -k "head or golden or long or whole" > gpurun_out/r04h2_tests.log 2>&1 || { tail -30 gpurun_out/r04h2_tests.log; exit 1; }
tail -2 gpurun_out/r04h2_tests.log
mkdir -p gpurun_out/r04h2p
SEPVAD_TAIL_PROBE=$PWD/gpurun_out/r04h2p/t timeout -k 10 200 python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline > gpurun_out/r04h2p/b.json 2>&1 || exit 1
python3 tools/tail_probe.py gpurun_out/r04h2p/t.tcnhead
timeout -k 10 800 bash tools/ab_bench.sh r04h2_bench 4 --steps 200 --warmup 20 -- sep-tfanet-vad_amd/libsepvad_base.so sep-tfanet-vad_amd/libsepvad_hrd8.so sep-tfanet-vad_amd/libsepvad.so
