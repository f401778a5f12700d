"""HBM traffic per launch of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

usage: python tools/pmc.py <fetch_dir> <write_dir> <kernel-substring> <out.json> [flops_or_bytes_note]

Corrections per /opt/skills/guides/MI355X_MICROARCH.md "HBM [CDNA4]": on gfx950 FETCH_SIZE reports
half the bytes of wide (16 B/lane) coalesced streaming reads -> doubled here; WRITE_SIZE is exact for
16-B-per-lane stores. Both counters are in KB (rocprofv3 derived metric) -> converted to bytes.
Infinity-Cache hits are counted by these memory-side counters (guide), so the figure is "bytes that
left the XCD L2s", an upper bound on HBM bytes.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, ksub):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if ksub not in r.get("Kernel_Name", ""):
                continue
            if r.get("Counter_Name") != counter:
                continue
            key = (f, r.get("Dispatch_Id"))
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    fd, wd, ksub, out = sys.argv[1:5]
    fetch = per_dispatch(fd, "FETCH_SIZE", ksub)
    write = per_dispatch(wd, "WRITE_SIZE", ksub)
    if not fetch or not write:
        raise SystemExit(f"kernel {ksub!r} not found (fetch {len(fetch)}, write {len(write)})")
    f_kb = sum(fetch) / len(fetch)
    w_kb = sum(write) / len(write)
    res = {
        "kernel": ksub,
        "dispatches": [len(fetch), len(write)],
        "fetch_size_kb_raw": f_kb,
        "write_size_kb_raw": w_kb,
        "read_bytes_per_launch": 2.0 * f_kb * 1024.0,
        "write_bytes_per_launch": w_kb * 1024.0,
        "hbm_bytes_per_launch": 2.0 * f_kb * 1024.0 + w_kb * 1024.0,
        "correction": "FETCH_SIZE x2 (gfx950 wide-read tally), KB->B; IC hits included (upper bound on HBM)",
    }
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
