"""ctypes front-end to oracle/liboracle_dw.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the plain-C CPU restatement of the reference's dynamic-wave
routing step (oracle/dw_oracle.c).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg import this module, and only as the checker.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle_dw.so")
REF_DIR = os.path.join(ORACLE_DIR, "_ref")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-C", ORACLE_DIR, "oracle"], check=True,
                           stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(LIB_PATH)
        L.orc_alloc.restype = ctypes.c_void_p
        L.orc_alloc.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_free.argtypes = [ctypes.c_void_p]
        L.orc_fd.restype = ctypes.POINTER(ctypes.c_double)
        L.orc_fd.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.orc_fi.restype = ctypes.POINTER(ctypes.c_int)
        L.orc_fi.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.orc_set_opt.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_double]
        L.orc_get_opt.restype = ctypes.c_double
        L.orc_get_opt.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.orc_prepare.argtypes = [ctypes.c_void_p]
        L.orc_routing_step.restype = ctypes.c_double
        L.orc_routing_step.argtypes = [ctypes.c_void_p, ctypes.c_double]
        L.orc_step.argtypes = [ctypes.c_void_p, ctypes.c_double]
        L.orc_xsect.restype = ctypes.c_double
        L.orc_xsect.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                ctypes.c_double, ctypes.c_double]
        _lib = L
    return _lib


# names shared by the reference dump (tests/_dumpio.py) and the oracle
NODE_STATIC_I = ["type", "degree", "outfallType", "outfallFlap"]
NODE_STATIC_D = ["invertElev", "fullDepth", "surDepth", "pondedArea", "crownElev",
                 "fullVolume", "fixedStage"]
NODE_STATE_D = ["newDepth", "oldDepth", "newVolume", "oldVolume", "inflow", "outflow",
                "newLatFlow", "oldLatFlow", "oldNetInflow", "oldFlowInflow", "overflow"]
LINK_STATIC_I = ["type", "node1", "node2", "hasFlapGate", "direction", "xtype",
                 "culvertCode", "barrels", "hasLosses"]
LINK_STATIC_D = ["offset1", "offset2", "qLimit", "cLossInlet", "cLossOutlet", "cLossAvg",
                 "seepRate", "yFull", "wMax", "ywMax", "aFull", "rFull", "sFull", "sMax",
                 "yBot", "aBot", "sBot", "rBot", "length", "modLength", "roughFactor",
                 "slope", "beta", "qMax", "setting"]
LINK_STATE_D = ["newFlow", "oldFlow", "newDepth", "oldDepth", "newVolume", "oldVolume",
                "a1", "a2", "q1", "q2"]
LINK_STATE_I = ["flowClass"]


class Oracle:
    """One network held by the C restatement."""

    def __init__(self, n_nodes: int, n_links: int, n_pollut: int = 0):
        self.L = lib()
        self.nN, self.nL, self.nP = n_nodes, n_links, n_pollut
        self.h = self.L.orc_alloc(n_nodes, n_links, n_pollut)

    def __del__(self):
        try:
            if self.h:
                self.L.orc_free(self.h)
        except Exception:
            pass

    def _n(self, name):
        if name.startswith("link."):
            n = self.nL
        elif name.startswith("pollut."):
            return max(self.nP, 1)
        else:
            n = self.nN
        if name in ("node.oldQual", "node.newQual", "node.qualIn", "link.oldQual",
                    "link.newQual"):
            n *= max(self.nP, 1)
        return n

    def d(self, name: str) -> np.ndarray:
        p = self.L.orc_fd(self.h, name.encode())
        if not p:
            raise KeyError(name)
        return np.ctypeslib.as_array(p, shape=(self._n(name),))

    def i(self, name: str) -> np.ndarray:
        p = self.L.orc_fi(self.h, name.encode())
        if not p:
            raise KeyError(name)
        return np.ctypeslib.as_array(p, shape=(self._n(name),))

    def opt(self, name: str, value: float):
        if self.L.orc_set_opt(self.h, name.encode(), float(value)) != 0:
            raise KeyError(name)

    def get(self, name: str) -> float:
        return self.L.orc_get_opt(self.h, name.encode())

    def prepare(self):
        rc = self.L.orc_prepare(self.h)
        if rc != 0:
            raise ValueError("network uses features outside the oracle's scope (%d)" % rc)

    def routing_step(self, fixed: float) -> float:
        return self.L.orc_routing_step(self.h, fixed)

    def step(self, dt: float) -> int:
        return self.L.orc_step(self.h, dt)

    def xsect(self, fn: int, link: int, x: float, x2: float = 0.0) -> float:
        return self.L.orc_xsect(self.h, fn, link, x, x2)


def oracle_from_dump(d: dict) -> Oracle:
    """Build an oracle network from a reference SWDUMP (static part + state after
    swmm_start)."""
    nn, nl, npol = (int(x) for x in d["counts"][:3])
    o = Oracle(nn, nl, npol)
    for k in NODE_STATIC_I:
        o.i("node." + k)[:] = d["node." + k]
    for k in NODE_STATIC_D + NODE_STATE_D:
        o.d("node." + k)[:] = d["node." + k]
    for k in LINK_STATIC_I:
        o.i("link." + k)[:] = d["link." + k]
    for k in LINK_STATIC_D + LINK_STATE_D:
        o.d("link." + k)[:] = d["link." + k]
    for k in LINK_STATE_I:
        o.i("link." + k)[:] = d["link." + k]
    od, oi = d["opt.d"], d["opt.i"]
    o.opt("routeStep", od[0])
    o.opt("courantFactor", od[1])
    o.opt("minRouteStep", od[2])
    o.opt("minSurfArea", od[3])
    o.opt("headTol", od[4])
    o.opt("crownCutoff", od[5])
    o.opt("evapRate", od[7])
    o.opt("maxTrials", oi[0])
    o.opt("surchargeMethod", oi[1])
    o.opt("inertDamping", oi[2])
    o.opt("normalFlowLtd", oi[3])
    o.opt("allowPonding", oi[4])
    if npol:
        o.d("pollut.kDecay")[:] = d["pollut.kDecay"]
    o.prepare()
    return o


def oracle_resume(d: dict) -> Oracle:
    """Oracle seeded from a mid-run engine dump (swmmx_exportState): the state
    of oracle_from_dump plus what persists across steps -- Xnode.oldSurfArea
    (surcharge denominator, dynwave.c:700, 728-729), Xnode.dYdT and the static
    VariableStep of the Courant step (dynwave.c:84, 209-218, 878-921)."""
    o = oracle_from_dump(d)
    for k in ("node.oldSurfArea", "node.dYdT", "link.froude"):
        if k in d:
            o.d(k)[:] = d[k]
    if o.nP:
        for k in ("node.newQual", "node.oldQual", "link.newQual", "link.oldQual"):
            if k in d:
                o.d(k)[:] = d[k]
    o.opt("variableStep", float(d["opt.d"][11]))
    return o
