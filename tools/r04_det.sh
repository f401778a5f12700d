# k_tcn16 determinism hypotheses (GPU box). usage: bash tools/r04_det.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04det}; out=gpurun_out/$tag; mkdir -p $out
run() { name=$1; shift; env "$@" timeout -k 10 200 python tools/det16.py $B $N > $out/det_$name.log 2>&1 || { tail -5 $out/det_$name.log; exit 1; }
        echo "== $name"; grep -E "sep:|vad:|capacity" $out/det_$name.log | sort | uniq -c | head -12; }
B=8 N=32000 run b8
B=64 N=32000 run b64_xmode1 SEPVAD_TCN_XMODE=1
B=64 N=32000 run b64_1percu SEPVAD_TCN16_DYNLDS=82000
B=64 N=8000 run b64_n8000
