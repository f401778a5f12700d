# Phase probes of the int8-lo k_tcn with the GEMM ring refills skipped (diag1) or the GEMM MFMAs skipped (diag2), one
# and two slices (diagnostics only: wrong results). usage: bash tools/r05_diag.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05diag}; mkdir -p $out
for lib in lib_final lib_diag1 lib_diag2; do for w in offline cfg5; do
  SEPVAD_TCN_WQ16=0 SEPVAD_LIB=$PWD/var/$lib.so SEPVAD_TCN_PROBE=$PWD/$out/p.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 100 --no-cpu-baseline --workload $w > $out/p.json 2> $out/p.err || exit 1
  python3 tools/tcn_probe.py $out/p.bin > $out/phases_${lib}_$w.txt && rm -f $out/p.bin || exit 1
  echo "== $lib $w"; sed -n 2p $out/phases_${lib}_$w.txt; grep -E "GEMM|update|moments|epilogue|dwconv" $out/phases_${lib}_$w.txt | head -6
done; done
