# Round 6: smoke + the tests new this round (fp32 long groups, two-slice other configs, cfg-1 CLI defaults, build id),
# then the headline bench (driver shape 20/5 and the steady window). usage: bash tools/r06_t1.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r06t}; out=gpurun_out/$tag; mkdir -p $out
step() { echo "== $1 $(date +%T)"; }
step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && tail -1 $out/smoke.log \
&& step pytest && timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_prep.py tests/test_gpu_parity.py -m gpu -x -v -s \
   --timeout 300 --timeout-method thread -k "fp32_gemms_long or other_configs or without_vad_defaults or native_library_is_loaded" > $out/pytest.log 2>&1; rc=$?
grep -E "passed|failed|error|build id" $out/pytest.log | tail -4; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit $rc; }
step bench20 && timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench20.json 2> $out/bench20.err && tail -1 $out/bench20.json | cut -c1-200 \
&& step bench && timeout -k 10 300 python3 bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err && tail -1 $out/bench.json | cut -c1-200
