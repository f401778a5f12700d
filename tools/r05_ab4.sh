# Static priority on the long-group and cfg 4 lines: var/lib_pit.so vs var/lib_prio.so, interleaved.
set -o pipefail
out=gpurun_out/${1:-r05u}; mkdir -p $out
for r in 1 2 3; do
  for lib in var/lib_pit.so var/lib_prio.so; do
    n=$(basename $lib .so)
    for w in "long --samples 960000 --batch 2" "cfg4"; do
      SEPVAD_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $w > $out/l.json 2> /dev/null || exit 1
      python3 -c "import json,sys; d=json.loads(open('$out/l.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$n', sys.argv[1], $r, d['value'], d['ms_per_step'], r.get('avg_launch_us'))" ${w%% *}
    done
  done
done | tee $out/lines.txt
