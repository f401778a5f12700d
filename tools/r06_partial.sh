# Partial-member penalty: cfg 2 at T = 126 (last member 30 valid frames) vs T = 128 (every member full), with and without
# the mask-free full-member loops (abl/lib_rs.so: RSRED only; abl/lib_rf.so: + FULLM). usage: bash tools/r06_partial.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p $out
for r in 1 2 3; do for n in rs rf; do for N in 32000 32512; do
  SEPVAD_LIB=$PWD/abl/lib_$n.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --samples $N > $out/l.json 2> $out/l.err || { tail -3 $out/l.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); print('$n N=$N', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done; done; done | tee $out/lines.txt
