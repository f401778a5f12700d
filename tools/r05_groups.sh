# All groups the chip holds (no multiple-of-8 rounding; the remainder groups span XCDs): cfg 3 streaming with and without
# SEPVAD_TCN_ALIGN8, cfg 5 with forced write-through hand-offs (the cross-XCD cost), and the bitwise digest of a
# 1792-window-like batch. usage: bash tools/r05_groups.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05g}; mkdir -p $out
step() { echo "== $1 $(date +%T)"; }
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], d['ms_per_step'], r.get('avg_launch_us'))" $1 $2; }
step digest && for a in 0 1; do SEPVAD_TCN_ALIGN8=$a SEPVAD_TCN_INFO=1 timeout -k 10 120 python3 tools/bitwise_ab.py 1200 48000 2>&1 | grep -E "k_tcn grid|libsepvad" | sort | uniq | tail -3 || exit 1; done | tee $out/digest.txt
for r in 1 2; do
  for a in 1 0; do
    SEPVAD_TCN_ALIGN8=$a timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload stream > $out/stream.$a.$r.json 2> $out/stream.$a.$r.err || exit 1
    line $out/stream.$a.$r.json "stream align8=$a round $r"
  done
done | tee $out/ab.txt
for x in 0 1; do
  SEPVAD_TCN_XMODE=$x timeout -k 10 200 python3 bench.py --no-cpu-baseline --workload cfg5 > $out/cfg5.x$x.json 2> /dev/null || exit 1
  line $out/cfg5.x$x.json "cfg5 xmode=$x"
done | tee -a $out/ab.txt
step done
