set -o pipefail
SEPVAD_LIB=$PWD/sep-tfanet-vad_amd/libsepvad_base.so timeout -k 10 200 python3 tools/diag_bf16.py run base > gpurun_out/diag_base.log 2>&1 || { tail -5 gpurun_out/diag_base.log; exit 1; }
timeout -k 10 200 python3 tools/diag_bf16.py run cur > gpurun_out/diag_cur.log 2>&1 || { tail -5 gpurun_out/diag_cur.log; exit 1; }
python3 tools/diag_bf16.py cmp base cur
