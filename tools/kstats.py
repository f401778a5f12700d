"""Print the per-kernel summary of one or more rocprofv3 --stats runs: tools/kstats.py <tag> [<tag> ...]"""
import csv
import sys

for tag in sys.argv[1:]:
    path = tag if tag.endswith(".csv") else f"gpurun_out/prof_{tag}/run_kernel_stats.csv"
    rows = list(csv.DictReader(open(path)))
    print(tag)
    for r in rows[:16]:
        print(f"  {r['Name'][:58]:58s} calls={r['Calls']:>5} avg={float(r['AverageNs'])/1000:8.2f}us"
              f" tot%={float(r['Percentage']):5.1f}")
