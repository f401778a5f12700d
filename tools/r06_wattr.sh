# Round 6, VERDICT r05 item 3: attribution of k_tcn's HBM-side writes. WRITE_SIZE per launch as the stack is truncated
# (SEPVAD_TCN_NBLK = 1, 6, 12, 24: the slope is the per-block hand-off traffic that leaves the L2s, the intercept the
# per-launch writes -- masks, VAD taps, spills), and with every hand-off forced write-through (SEPVAD_TCN_XMODE=1), at
# cfg 2 (one slice), cfg 5 (two slices) and 60 s files (G = 118, cross-XCD groups).
# usage: bash tools/r06_wattr.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r06w}; out=$PWD/gpurun_out/$tag; mkdir -p $out
run() {  # name, env, bench args
  local n=$1 e=$2; shift 2
  env $e timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/$n -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $out/$n.log 2>&1 || { echo "FAIL $n"; tail -3 $out/$n.log; return 1; }
  python3 - $out/$n $n <<'PY'
import sys; sys.path.insert(0, 'tools')
from pmc import per_dispatch
v = per_dispatch(sys.argv[1], "WRITE_SIZE", "k_tcn<")
v.sort()
print(f"{sys.argv[2]:28s} k_tcn WRITE_SIZE per launch (MB): median {v[len(v)//2]*1024/1e6:8.2f}  n={len(v)}")
PY
}
for w in "cfg2:--workload offline" "cfg5:--workload cfg5" "long60:--workload long --samples 960000 --batch 2"; do
  wn=${w%%:*}; wa=${w#*:}
  for nb in 1 6 12 24; do run ${wn}_nblk$nb "SEPVAD_TCN_NBLK=$nb" $wa || exit 1; done
  run ${wn}_xmode1 "SEPVAD_TCN_XMODE=1" $wa || exit 1
done | tee $out/summary.txt
