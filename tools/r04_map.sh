# k_tcn16: does the failure need two members of one group on a CU? (SEPVAD_TCN_XMODE=2 interleaves groups)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r04m}; mkdir -p $out
for w in 8 4; do
  for xm in 2 0; do
    SEPVAD_TCN_XMODE=$xm SEPVAD_TCN16_WAVES=$w timeout -k 10 200 python tools/det16.py 64 32000 > $out/det_w${w}_x$xm.log 2>&1 || { tail -5 $out/det_w${w}_x$xm.log; exit 1; }
    echo "== waves $w xmode $xm"; grep -E "run . sep|k_tcn16 vs k_tcn sep" $out/det_w${w}_x$xm.log
  done
done
SEPVAD_TCN_XMODE=2 SEPVAD_TCN16=1 SEPVAD_TCN_PROBE=$PWD/$out/probe_x2.bin timeout -k 10 120 python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 && python3 tools/tcn_probe.py $out/probe_x2.bin pairs | tail -4
