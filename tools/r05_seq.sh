# Batched member sums + parallel XCD check: bitwise digests against the previous library (var/lib_base.so) at cfg 2,
# cfg 5, 16 s and 60 s files; alternating 60 s / cfg 2 bench A/B; the fused suite. usage: bash tools/r05_seq.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05s}; mkdir -p $out
export SEPVAD_VAD_LABEL_LOG=$out/vad_labels.txt
step() { echo "== $1 $(date +%T)"; }
step digests
for bn in "64 32000" "128 32000" "8 256000" "2 960000"; do
  for lib in var/lib_base.so sep-tfanet-vad_amd/libsepvad.so; do
    SEPVAD_LIB=$PWD/$lib timeout -k 10 120 python3 tools/bitwise_ab.py $bn 2>/dev/null | tail -1 || exit 1
  done
done | tee $out/digests.txt
step ab
for r in 1 2 3; do
  for lib in var/lib_base.so sep-tfanet-vad_amd/libsepvad.so; do
    n=$(basename $(dirname $lib))
    SEPVAD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload long --samples 960000 --batch 2 > $out/l60.$n.$r.json 2> /dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$out/l60.$n.$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('long60 $n $r', d['value'], d['ms_per_step'], r.get('avg_launch_us'))"
  done
done | tee $out/ab.txt
step pytest && timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $out/pytest.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit $rc; }
step done
