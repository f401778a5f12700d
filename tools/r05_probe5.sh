# Two-slice phase probe (cfg 5) and a kernel trace of the cfg 2 bench (inter-kernel gaps). usage: bash tools/r05_probe5.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05p5}; mkdir -p $out
SEPVAD_TCN_PROBE=$PWD/$out/probe_cfg5.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --workload cfg5 > $out/p5.json 2> $out/p5.err \
&& python3 tools/tcn_probe.py $out/probe_cfg5.bin > $out/phases_cfg5.txt && rm -f $out/probe_cfg5.bin \
&& timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $out/trace.log 2>&1 \
&& cat $out/phases_cfg5.txt
