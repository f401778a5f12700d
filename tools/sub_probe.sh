# Sub-phase probe with a variant library (tools/build_variants.sh <name>="-DTCN_SUB=1").
# usage: bash tools/sub_probe.sh <tag> <variant-name> <TCN_SUB value>
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
SEPVAD_LIB=$PWD/var/lib_$2.so SEPVAD_TCN_PROBE=$PWD/$out/probe_$2.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 2 \
    --no-cpu-baseline > $out/bp_$2.json 2> $out/bp_$2.err \
&& TCN_SUB=$3 python3 tools/tcn_probe.py $out/probe_$2.bin > $out/phases_$2.txt && cat $out/phases_$2.txt
