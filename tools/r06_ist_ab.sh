timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fused.py -k "vad or golden or side or istft or est" > gpurun_out/r06ist_tests.txt 2>&1; tail -3 gpurun_out/r06ist_tests.txt
KSTEPS=300 bash tools/kstat_ab.sh r06istk abl/lib_prev.so abl/lib_ist.so abl/lib_prev.so abl/lib_ist.so
bash tools/r06_lines4.sh r06istl 2 prev ist
