# Bitwise digests (even/odd T, N % 4 != 0) and k_istft_pair stats of two libraries. usage: bash tools/r05_istw.sh <tag> libA libB
set -o pipefail
export TMPDIR=/tmp
tag=$1; A=$2; B=$3; out=gpurun_out/$tag; mkdir -p $out
for bn in "64 32000" "64 32001" "64 31900" "3 48002" "1 16000"; do
  for lib in $A $B; do SEPVAD_LIB=$PWD/$lib timeout -k 10 120 python3 tools/bitwise_ab.py $bn 2>/dev/null | tail -1 || exit 1; done
done | tee $out/digests.txt
for lib in $A $B; do
  n=$(basename $lib .so)
  SEPVAD_LIB=$PWD/$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/prof_$n -o run -- python3 bench.py --no-cpu-baseline --steps 40 --warmup 10 > $out/l_$n.json 2> /dev/null || exit 1
  f=$(find $out/prof_$n -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$n" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("k_istft", "k_tcn", "k_stft", "k_vad")):
        print(sys.argv[2], r["Name"][:40], r["Calls"], r["AverageNs"])
PY
  python3 -c "import json; d=json.loads(open('$out/l_$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'])"
done | tee $out/stats.txt
find $out -name '*.csv' ! -name '*kernel_stats.csv' -delete
