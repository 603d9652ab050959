"""HBM bytes per launch of a kernel from two separate rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE; counter_collection.csv), corrected as MI355X_MICROARCH.md
§HBM prescribes: FETCH_SIZE (KB) x 1024 x 2 (gfx950 counts half of a 16-B/lane
streaming read) + WRITE_SIZE (KB) x 1024.  Writes/updates profiles/traffic.json.

    python scripts/pmc_traffic.py NAME KERNEL_SUBSTR FETCH.csv WRITE.csv OUT_FETCH OUT_WRITE"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


COLS = ["Dispatch_Id", "Kernel", "Grid_Size", "Workgroup_Size", "VGPR_Count", "SGPR_Count",
        "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]


def per_launch(path, counter, sub, out_path):
    """Mean counter value per launch of the kernels matching sub; the matching rows are
    written (trimmed to COLS) to out_path."""
    vals, kern, rows = [], None, []
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel", row.get("Kernel_Name"))
            if row["Counter_Name"] == counter and sub in name:
                vals.append(float(row["Counter_Value"]))
                kern = name
                rows.append({c: (name if c == "Kernel" else row.get(c, "")) for c in COLS})
    with open(out_path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=COLS)
        w.writeheader()
        w.writerows(rows)
    return sum(vals) / len(vals), len(vals), kern


def main():
    name, sub, fetch_csv, write_csv, out_f, out_w = sys.argv[1:7]
    fkb, nf, kern = per_launch(fetch_csv, "FETCH_SIZE", sub, os.path.join(ROOT, out_f))
    wkb, nw, _ = per_launch(write_csv, "WRITE_SIZE", sub, os.path.join(ROOT, out_w))
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
