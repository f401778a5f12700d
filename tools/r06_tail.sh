# Round 6: tail probes (k_stft_gate, k_tcn's output head, k_istft_pair) at cfg 2 after a 300-forward warm-up.
# usage: bash tools/r06_tail.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r06tail}; mkdir -p $out
SEPVAD_TAIL_PROBE=$PWD/$out/t timeout -k 10 120 python3 bench.py --steps 2 --warmup 300 --no-cpu-baseline > $out/t.json 2> $out/t.err || { tail -3 $out/t.err; exit 1; }
ls $out
for k in stft tcnhead istft; do [ -f $out/t.$k ] && { echo "== $k"; python3 tools/tail_probe.py $out/t.$k 2.1; }; done | tee $out/tail.txt
rm -f $out/t.stft $out/t.tcnhead $out/t.istft $out/t.vad1 $out/t.head
