# k_tcn16 vs k_tcn on a truncated stack (SEPVAD_TCN_NBLK), B=64 N=32000 (two workgroups per CU). usage: bash tools/r04_det3.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04det3}; out=gpurun_out/$tag; mkdir -p $out
run() { name=$1; shift; env "$@" timeout -k 10 200 python tools/det16.py $B $N > $out/det_$name.log 2>&1 || { tail -5 $out/det_$name.log; exit 1; }
        echo "== $name"; grep -E "run 1 sep|run 2 sep|k_tcn16 vs k_tcn sep" $out/det_$name.log | head -12; }
for nb in 1 2 3; do B=64 N=32000 run nb$nb SEPVAD_TCN_NBLK=$nb; done
B=32 N=32000 run b32
B=256 N=8000 run b256_n8000
B=128 N=16000 run b128_n16000
