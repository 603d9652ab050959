"""HBM bytes per launch of a kernel from two separate rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE; counter_collection.csv), corrected as MI355X_MICROARCH.md
§HBM prescribes: FETCH_SIZE (KB) x 1024 x 2 (gfx950 counts half of a 16-B/lane
streaming read) + WRITE_SIZE (KB) x 1024.  Writes/updates profiles/traffic.json.

    python scripts/pmc_traffic.py NAME KERNEL_SUBSTR FETCH.csv WRITE.csv OUT_FETCH OUT_WRITE"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, counter, sub):
    vals, kern = [], None
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter and sub in row["Kernel"]:
                vals.append(float(row["Counter_Value"]))
                kern = row["Kernel"]
    return sum(vals) / len(vals), len(vals), kern


def main():
    name, sub, fetch_csv, write_csv, out_f, out_w = sys.argv[1:7]
    fkb, nf, kern = per_launch(fetch_csv, "FETCH_SIZE", sub)
    wkb, nw, _ = per_launch(write_csv, "WRITE_SIZE", sub)
    shutil.copy(fetch_csv, os.path.join(ROOT, out_f))
    shutil.copy(write_csv, os.path.join(ROOT, out_w))
    path = os.path.join(ROOT, "profiles", "traffic.json")
    t = json.load(open(path)) if os.path.exists(path) else {}
    t[name] = dict(hbm_bytes_per_launch=fkb * 1024 * 2 + wkb * 1024, fetch_size_kb=fkb,
                   write_size_kb=wkb, fetch_bytes_corrected=fkb * 1024 * 2, write_bytes=wkb * 1024,
                   correction="FETCH_SIZE(KB)*1024*2 (gfx950 half-count of 16-B/lane streams, "
                              "MI355X_MICROARCH.md HBM) + WRITE_SIZE(KB)*1024",
                   kernel=kern, launches=min(nf, nw),
                   source=f"{out_f}, {out_w} (separate rocprofv3 --pmc passes)")
    json.dump(t, open(path, "w"), indent=1)
    print(json.dumps(t[name]))


if __name__ == "__main__":
    main()
