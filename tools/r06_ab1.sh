# Round 6 A/B 1: bitwise digests + k_tcn cycles of the a1 / widening-pipeline / one-slice fp16-lo variants (cfg 2).
# usage: bash tools/r06_ab1.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r06a}; out=gpurun_out/$tag; mkdir -p $out
step() { echo "== $1 $(date +%T)"; }
step digests
for spec in base a1v wpipe both base@SEPVAD_TCN_WQ16=2; do
  lib=${spec%%@*}; envs=""; [ "$spec" != "$lib" ] && envs=${spec#*@}
  for bn in "64 32000" "128 32000"; do
    env $envs SEPVAD_LIB=$PWD/abl/lib_$lib.so timeout -k 10 120 python3 tools/bitwise_ab.py $bn || exit 1
  done
done | tee $out/digests.txt
step cycles
bash tools/ab_cyc.sh $tag/cyc 4 300 abl/lib_base.so abl/lib_a1v.so abl/lib_wpipe.so abl/lib_both.so abl/lib_base.so@SEPVAD_TCN_WQ16=2 abl/lib_both.so@SEPVAD_TCN_WQ16=2 > $out/cyc.log 2>&1 || exit 1
tail -7 $out/cyc.log
