# Long-file VAD features (k_vad_feat_rec): the whole-file fused tests, the 60 s line, kernel stats; the tail probe of cfg 2.
# usage: bash tools/r05_long.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05l}; mkdir -p $out
export SEPVAD_VAD_LABEL_LOG=$out/vad_labels.txt
step() { echo "== $1 $(date +%T)"; }
step pytest && timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_boundary.py -m gpu -x -v --timeout 240 --timeout-method thread -k "whole_file or long" > $out/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $out/pytest.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit $rc; }
step long60 && timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload long --samples 960000 --batch 2 > $out/long60.json 2> $out/long60.err \
&& tail -1 $out/long60.json | cut -c1-200 \
&& step long60_prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof60 -o run -- python3 bench.py --no-cpu-baseline --workload long --samples 960000 --batch 2 --steps 10 --warmup 2 > $out/prof60.log 2>&1 \
&& python3 tools/kstats.py $(find $out/prof60 -name "*kernel_stats.csv" | head -1) \
&& step tail && bash tools/tail_round.sh ${1:-r05l}/tail > /dev/null && cat $out/tail/stft_phases.txt $out/tail/istft_phases.txt \
&& step done
