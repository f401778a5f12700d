# Round 6 A/B of abl/lib_<name>.so variants (fused_x3l2 object only): bitwise digests at cfg 2 (one slice) and cfg 5
# (two slices, int8 kernel: SEPVAD_TCN_WQ16=0), then interleaved k_tcn cycles at cfg 2 (tools/ab_cyc.sh).
# usage: bash tools/r06_ab.sh <tag> <rounds> name1 name2 ...
set -o pipefail
export TMPDIR=/tmp
tag=$1; R=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
echo "== digests $(date +%T)"
for n in "$@"; do
  SEPVAD_LIB=$PWD/abl/lib_$n.so timeout -k 10 120 python3 tools/bitwise_ab.py 64 32000 2>/dev/null | grep lib_ || exit 1
  SEPVAD_TCN_WQ16=0 SEPVAD_LIB=$PWD/abl/lib_$n.so timeout -k 10 120 python3 tools/bitwise_ab.py 128 32000 2>/dev/null | grep lib_ || exit 1
done | tee $out/digests.txt
echo "== cycles $(date +%T)"
libs=""; for n in "$@"; do libs="$libs abl/lib_$n.so"; done
bash tools/ab_cyc.sh $tag/cyc $R 300 $libs > $out/cyc.log 2>&1 || { tail -5 $out/cyc.log; exit 1; }
tail -$# $out/cyc.log
