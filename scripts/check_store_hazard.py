"""Static check of the gfx950 store-data hazard in hipcc's output: a dwordx3/x4 VMEM store
whose data VGPRs a VALU instruction overwrites within the next two instructions
(the store may read the new value).  python scripts/check_store_hazard.py file.s ..."""
import re
import sys

STORE = re.compile(r"^\s*(global|buffer|flat|scratch)_store_dwordx[34]\s+(?:v\[?(\d+)(?::(\d+))?\]?,\s*)?")
VALU = re.compile(r"^\s*(v_[a-z0-9_]+)\s+v\[?(\d+)(?::(\d+))?\]?")


def regs(lo, hi):
    return set(range(int(lo), int(hi if hi else lo) + 1))


def main():
    bad = 0
    for path in sys.argv[1:]:
        fn = None
        lines = open(path).read().splitlines()
        insts = []  # (line no, text, function)
        for i, ln in enumerate(lines):
            if re.match(r"^_Z\w+:", ln):
                fn = ln[:-1]
            t = ln.split(";")[0].strip()
            if t and not t.endswith(":") and not t.startswith("."):
                insts.append((i + 1, t, fn))
        for k, (no, t, fn) in enumerate(insts):
            m = re.match(r"^(global|buffer|flat|scratch)_store_dwordx([34])\s+(\S+)", t)
            if not m:
                continue
            data = m.group(3).rstrip(",")
            if "[" in data:
                lo, hi = re.match(r"v\[(\d+):(\d+)\]", data).groups()
            else:
                continue
            if m.group(1) == "global" or m.group(1) == "flat":
                # global_store_dwordx4 vaddr, vdata, ...: data is the second operand
                ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
                mm = re.match(r"v\[(\d+):(\d+)\]", ops[1])
                if not mm:
                    continue
                lo, hi = mm.groups()
            r = regs(lo, hi)
            for j in range(1, 3):
                if k + j >= len(insts):
                    break
                nt = insts[k + j][1]
                if nt.startswith("s_nop"):
                    break
                v = VALU.match(nt)
                if v and regs(v.group(2), v.group(3)) & r:
                    print(f"{path}:{no}: {fn}: '{t}' then '{nt}'")
                    bad += 1
                    break
    print(f"{bad} hazard(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
