"""A/B bitwise check of two engine builds (diagnostic): run each case's
golden input with the library named on the command line and write its
binary results; the caller compares the files.
  python tools/ab_bitwise.py <lib.so> <out_dir> case...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stormwater-management-model_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import swmm5      # noqa: E402
import _golden    # noqa: E402

lib, outdir = sys.argv[1], sys.argv[2]
os.makedirs(outdir, exist_ok=True)
eng = swmm5.SWMM(lib)
for name in sys.argv[3:]:
    rc = eng.run(_golden.inp(name), os.path.join(outdir, name + ".rpt"), os.path.join(outdir, name + ".out"))
    print(name, rc)
