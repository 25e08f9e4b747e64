"""Known-answer vectors for the cross-section relations, from the reference.

TEST INFRASTRUCTURE ONLY -- needs the reference build (oracle/_ref, made from
/root/reference by `make -C oracle ref`); run in the survey container:

    python tests/golden/make_xsect_kat.py

For every shape case in _xsect_cases.SHAPES it calls the reference's own
xsect_setParams and xsect_getAofY / WofY / RofY / YofA / RofA / SofA / AofS /
dSdA / Ycrit (xsect.c:216-1319) through ctypes on a fresh section per point
(FILLED_CIRCULAR evaluations modify the section in place) and stores inputs
and outputs in xsect_kat.npz.
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from _xsect_cases import SHAPES, FUNCS, points  # noqa: E402

REF = os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle", "_ref", "libswmm5_ref.so")


class TXsect(ctypes.Structure):           # objects.h:581-599
    _fields_ = [("type", ctypes.c_int), ("culvertCode", ctypes.c_int), ("transect", ctypes.c_int)] + \
               [(n, ctypes.c_double) for n in ("yFull", "wMax", "ywMax", "aFull", "rFull", "sFull",
                                             "sMax", "yBot", "aBot", "sBot", "rBot")]


PARAMS = ("yFull", "wMax", "ywMax", "aFull", "rFull", "sFull", "sMax", "yBot", "aBot", "sBot", "rBot")


def ref_lib():
    L = ctypes.CDLL(REF)
    for f in ("xsect_getAofY", "xsect_getWofY", "xsect_getRofY", "xsect_getYofA", "xsect_getRofA",
              "xsect_getSofA", "xsect_getAofS", "xsect_getdSdA", "xsect_getYcrit"):
        getattr(L, f).restype = ctypes.c_double
        getattr(L, f).argtypes = [ctypes.POINTER(TXsect), ctypes.c_double]
    L.xsect_setParams.argtypes = [ctypes.POINTER(TXsect), ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                  ctypes.c_double]
    return L


def make_section(L, code, p):
    x = TXsect()
    arr = (ctypes.c_double * 4)(*p)
    assert L.xsect_setParams(ctypes.byref(x), code, arr, 1.0) == 1
    return x


def main():
    L = ref_lib()
    out = {}
    for k, (name, code, p) in enumerate(SHAPES):
        x0 = make_section(L, code, p)
        par = np.array([getattr(x0, n) for n in PARAMS])
        out["params_%d" % k] = par
        for fi, fname in enumerate(FUNCS, start=1):
            xs = points(fi, dict(zip(PARAMS, par)))
            f = getattr(L, "xsect_get" + fname)
            ys = np.array([f(ctypes.byref(make_section(L, code, p)), v) for v in xs])
            out["x_%d_%d" % (k, fi)] = xs
            out["y_%d_%d" % (k, fi)] = ys
    np.savez_compressed(os.path.join(HERE, "xsect_kat.npz"), **out)
    print("xsect_kat.npz:", len(SHAPES), "sections")


if __name__ == "__main__":
    main()
