# Round 6: phase probes of the current k_tcn (cfg 2 one slice, cfg 5 two slices) after a 300-forward warm-up, then
# interleaved cfg 2 lines with the VAD features in k_vad_feat (SEPVAD_VAD_FEAT=1, default) or inside k_istft_pair (0).
# usage: bash tools/r06_probe_vf.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r06pv}; mkdir -p $out
step() { echo "== $1 $(date +%T)"; }
step probe_cfg2 && SEPVAD_TCN_PROBE=$PWD/$out/probe_cfg2.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 300 --no-cpu-baseline > $out/p2.json 2> $out/p2.err \
&& python3 tools/tcn_probe.py $out/probe_cfg2.bin > $out/phases_cfg2.txt && head -20 $out/phases_cfg2.txt \
&& step probe_cfg5 && SEPVAD_TCN_PROBE=$PWD/$out/probe_cfg5.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 150 --no-cpu-baseline --workload cfg5 > $out/p5.json 2> $out/p5.err \
&& python3 tools/tcn_probe.py $out/probe_cfg5.bin > $out/phases_cfg5.txt && head -20 $out/phases_cfg5.txt \
&& step vadfeat && for r in 1 2 3; do for vf in 1 0; do
  SEPVAD_VAD_FEAT=$vf timeout -k 10 200 python3 bench.py --no-cpu-baseline > $out/l.json 2> $out/l.err || { tail -3 $out/l.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); print('vad_feat=$vf', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done; done | tee $out/vadfeat_lines.txt
