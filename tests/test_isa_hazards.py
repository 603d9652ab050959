"""The gfx950 ISA hipcc emits for every kernel has no dwordx3/x4 store whose data
registers a VALU overwrites within two instructions (measured on MI355X: such a store
may write the new value — nondeterministic sort output until k_bitonic.hip fenced its
16-B stores with s_nop 1).  CPU-only: compiles to .s (make asm) and scans it."""
import glob
import os
import subprocess
import sys

from conftest import ROOT


def test_no_store_data_hazard():
    pkg = os.path.join(ROOT, "fl-tee_amd")
    subprocess.run(["make", "-s", "-j8", "-C", pkg, "asm"], check=True, capture_output=True)
    files = sorted(glob.glob(os.path.join(pkg, "build", "*.s")))
    assert files
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_store_hazard.py"), *files],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
