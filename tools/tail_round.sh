# Tail-kernel phase probes (k_stft_gate, k_istft_pair) of one forward. usage: bash tools/tail_round.sh <tag>
set -o pipefail
out=gpurun_out/${1:-tail}; mkdir -p $out
SEPVAD_TAIL_PROBE=$PWD/$out/tp timeout -k 10 120 python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline > $out/tp.json 2> $out/tp.err \
&& python3 tools/tail_probe.py $out/tp.stft > $out/stft_phases.txt && python3 tools/tail_probe.py $out/tp.istft > $out/istft_phases.txt \
&& python3 tools/tail_probe.py $out/tp.head > $out/head_phases.txt \
&& cat $out/stft_phases.txt $out/head_phases.txt $out/istft_phases.txt
{ [ -f $out/tp.vad1 ] && python3 tools/tail_probe.py $out/tp.vad1; } || true
