set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pyt_u.log 2>&1; tail -2 gpurun_out/pyt_u.log
bash tools/sub_probe.sh r02u sub1 1 | tail -4 && bash tools/ab.sh r02u 4 var/lib_pfx0.so var/lib_pfx1.so | tail -2
