# Inter-forward gaps of the cfg 2 bench (kernel trace) with and without the per-forward `done` event record, and lines.
# usage: bash tools/r05_gap.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05gap}; mkdir -p $out
for v in 0 1; do
  SEPVAD_DIAG_NO_DONE=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/t$v -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $out/t$v.log 2>&1 || exit 1
  python3 - $out/t$v/run_kernel_trace.csv $v <<'PY'
import csv, sys, statistics
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
g, prev = [], None
for r in rows:
    if prev is not None and 'k_stft_gate' in r['Kernel_Name'] and 'k_istft' in prev['Kernel_Name']:
        g.append((int(r['Start_Timestamp']) - int(prev['End_Timestamp'])) / 1e3)
    prev = r
print('no_done', sys.argv[2], 'gaps', [round(x, 1) for x in g[:24]])
PY
done
for r in 1 2; do for v in 0 1; do
  SEPVAD_DIAG_NO_DONE=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline > $out/l.json 2> /dev/null || exit 1
  python3 -c "import json; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); print('no_done $v', d['value'], d['ms_per_step'])"
done; done
find $out -name '*.csv' -delete
