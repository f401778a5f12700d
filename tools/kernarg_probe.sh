# k_tcn prologue diagnostics: phase probe of a cold launch and of a launch right after an unprobed one
set -o pipefail
out=gpurun_out/${1:-r02o}; mkdir -p $out
SEPVAD_TCN_PROBE=$PWD/$out/probe_cold.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline > $out/bp.json 2> $out/bp.err \
&& python3 tools/tcn_probe.py $out/probe_cold.bin > $out/phases_cold.txt && head -6 $out/phases_cold.txt \
&& SEPVAD_TCN_PROBE_WARM=1 SEPVAD_TCN_PROBE=$PWD/$out/probe_warm.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline > $out/bp2.json 2> $out/bp2.err \
&& python3 tools/tcn_probe.py $out/probe_warm.bin > $out/phases_warm.txt && head -6 $out/phases_warm.txt
