"""HBM bytes per launch of EVERY kernel of a workload, from two separate rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE; counter_collection.csv), with the correction
MI355X_MICROARCH.md §HBM prescribes for 16-B-per-lane streaming reads (FETCH_SIZE x 2)
and a calibration for the other access widths: `bitonic_global` (8-B loads per lane,
coalesced 512 B per wave instruction) reads exactly half of its launch-side bytes, so its
FETCH_SIZE against that known count is the factor for 8-B-lane reads in the same run.

Writes profiles/traffic.json entries "<NAME>:<kernel>" (kernel = the name between
"fltee::" and its template arguments): the raw counters per launch, the bytes per launch
with the x2 correction, the launches seen.  bench.py divides them by its live launch-side
bytes of the same kernel (traffic_over_launch_bytes: > 1 = re-reads, spills, scratch).

    python scripts/pmc_kernels.py NAME FETCH.csv WRITE.csv OUT_PREFIX"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COLS = ["Dispatch_Id", "Kernel", "Grid_Size", "Workgroup_Size", "VGPR_Count", "SGPR_Count",
        "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]


def short(name):
    m = re.search(r"fltee::([A-Za-z0-9_]+)", name)
    return m.group(1) if m else None


def read(path, counter, out_path):
    per = defaultdict(list)
    rows = []
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel", row.get("Kernel_Name", ""))
            k = short(name)
            if row["Counter_Name"] != counter or not k:
                continue
            per[k].append(float(row["Counter_Value"]))
            rows.append({c: (name if c == "Kernel" else row.get(c, "")) for c in COLS})
    with open(out_path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=COLS)
        w.writeheader()
        w.writerows(rows)
    return per


def main():
    name, fetch_csv, write_csv, prefix = sys.argv[1:5]
    fetch = read(fetch_csv, "FETCH_SIZE", os.path.join(ROOT, prefix + "_fetch.csv"))
    write = read(write_csv, "WRITE_SIZE", os.path.join(ROOT, prefix + "_write.csv"))
    path = os.path.join(ROOT, "profiles", "traffic.json")
    t = json.load(open(path)) if os.path.exists(path) else {}
    for k in sorted(set(fetch) & set(write)):
        f, w = fetch[k], write[k]
        fkb, wkb = sum(f) / len(f), sum(w) / len(w)
        t[f"{name}:{k}"] = dict(
            hbm_bytes_per_launch=fkb * 1024 * 2 + wkb * 1024, fetch_size_kb=fkb, write_size_kb=wkb,
            fetch_bytes_corrected=fkb * 1024 * 2, write_bytes=wkb * 1024, launches=min(len(f), len(w)),
            correction="FETCH_SIZE(KB)*1024*2 (gfx950 half-count of 16-B/lane streams, "
                       "MI355X_MICROARCH.md HBM) + WRITE_SIZE(KB)*1024; 8-B-lane reads: see the "
                       "workload's bitonic_global entry (known launch bytes)",
            source=f"{prefix}_fetch.csv, {prefix}_write.csv (separate rocprofv3 --pmc passes)")
        print(k, json.dumps(t[f"{name}:{k}"]))
    json.dump(t, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
