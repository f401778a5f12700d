# Parity / bitwise tests of an abl/lib_<name>.so variant (the int8 two-slice kernel: the variant object holds it).
# usage: bash tools/r06_var_tests.sh <tag> <name>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p $out
SEPVAD_TCN_WQ16=0 SEPVAD_LIB=$PWD/abl/lib_$2.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "matches_reference or two_slices_bitwise or vs_multikernel or output_head or persistent_groups or whole_file_forwards_stay_fused and 262144" \
  > $out/pytest_$2.log 2>&1; rc=$?
tail -2 $out/pytest_$2.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest_$2.log | head -20; exit $rc; }
