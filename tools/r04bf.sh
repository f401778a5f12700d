set -o pipefail
for lib in libsepvad; do
  SEPVAD_LIB=$PWD/sep-tfanet-vad_amd/$lib.so timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_precision.py -k "tolerance and cfg2" -s > gpurun_out/r04bf_$lib.log 2>&1
  echo "$lib rc=$?"; grep -o '{"arm".*}' gpurun_out/r04bf_$lib.log | python3 -c "
import sys, json
for l in sys.stdin:
    d=json.loads(l); print(d['arm'], 'sep', '%.2e'%d['sep_maxabs'], 'flips', d['vad_flips'], 'vadp', '%.2e'%d['vad_prob_maxabs'])"
done
