"""Per-kernel SQ/SQC counter summary from the rocprofv3 --pmc passes of
scripts/gpu_evidence.sh (SQ=...): averages per dispatch, with the derived figures used in
DESIGN.md (VALU / SALU / LDS busy share of the dispatch's cycles per SIMD or CU).

    python scripts/sq_summary.py gpurun_out/<TAG> c5 [kernel-substring ...]"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def load(out, w):
    res = defaultdict(lambda: defaultdict(list))
    for p in ("sq1", "sq2", "sq3", "sqc"):
        for f in glob.glob(f"{out}/{p}_{w}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r.get("Kernel_Name", r.get("Kernel", ""))
                m = re.search(r"fltee::([a-z_]+(<[^>]*>)?)", k)
                if m:
                    res[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return res


def main():
    out, w = sys.argv[1], sys.argv[2]
    subs = sys.argv[3:]
    res = load(out, w)
    rows = {}
    for kn, c in res.items():
        if subs and not any(s in kn for s in subs):
            continue
        avg = {k: sum(v) / len(v) for k, v in c.items()}
        rows[kn] = avg
        print(kn)
        print("   ", json.dumps({k: float(f"{v:.4g}") for k, v in sorted(avg.items())}))
    return rows


if __name__ == "__main__":
    main()
