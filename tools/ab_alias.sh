set -o pipefail
bash tools/kstat_ab.sh r02aq var/lib_alias0.so var/lib_alias1.so && SEPVAD_LIB=$PWD/var/lib_alias0.so SEPVAD_TAIL_PROBE=$PWD/gpurun_out/r02aq/tp timeout -k 10 120 python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline > gpurun_out/r02aq/tp.json 2>/dev/null && python3 tools/tail_probe.py gpurun_out/r02aq/tp.head
