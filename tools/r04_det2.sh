# k_tcn16 determinism bisection (GPU box). usage: bash tools/r04_det2.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04det2}; out=gpurun_out/$tag; mkdir -p $out
run() { name=$1; shift; env "$@" SEPVAD_TCN_INFO=1 timeout -k 10 200 python tools/det16.py $B $N > $out/det_$name.log 2>&1 || { tail -5 $out/det_$name.log; exit 1; }
        echo "== $name"; grep -E "run 1 sep|k_tcn16 vs k_tcn sep|k_tcn16 grid" $out/det_$name.log | sort | uniq -c | head -12; }
B=32 N=32000 run b32
B=128 N=8000 run b128_n8000
B=256 N=8000 run b256_n8000
B=64 N=32000 run b64_dyn4k SEPVAD_TCN16_DYNLDS=4000
B=128 N=16000 run b128_n16000
