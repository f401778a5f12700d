# Boundary tests (stream contexts, eviction) and interleaved cfg 2 / cfg 3 lines without the per-forward event record.
# usage: bash tools/r05_nodone.sh <tag> <previous lib>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05nd}; prev=$2; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_boundary.py -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $out/pytest.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit $rc; }
for r in 1 2 3; do for lib in $prev sep-tfanet-vad_amd/libsepvad.so; do for w in offline stream; do
  SEPVAD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload $w > $out/l.json 2> /dev/null || exit 1
  python3 -c "import json; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); print('$(basename $lib .so) $w', d['value'], d['ms_per_step'])"
done; done; done | tee $out/lines.txt
