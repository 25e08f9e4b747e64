"""Golden-fixture helpers (test infrastructure only)."""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
CASES = ["grid12", "grid12_var_qual", "grid10_surcharge", "example", "example_var",
         "example_qual"]
# DWF-only networks: lateral inflow is constant and pollutant loads are
# q * concentration, so the oracle can be fed without the inflow machinery
DWF_ONLY = {"grid12", "grid12_var_qual", "grid10_surcharge"}
GRID_CONC = [5.0, 10.0, 15.0, 20.0, 25.0, 30.0]


def load(name: str) -> dict:
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def inp(name: str) -> str:
    return os.path.join(GOLDEN, name + ".inp")


def ref_out(name: str) -> bytes:
    return np.load(os.path.join(GOLDEN, name + ".ref_out.npy"), allow_pickle=False).tobytes()


def every(d: dict) -> int:
    return int(d["s.every"][0])


def grid_qual_loads(d: dict, lat: np.ndarray) -> np.ndarray:
    """Pollutant mass loads of one step, in addDryWeatherInflows' arithmetic
    order (routing.c:540-572): w = q*cDWF; w += q*c; w -= q*cDWF."""
    P = int(d["counts"][2])
    out = np.zeros((P, lat.size))
    for p in range(P):
        dc = d["pollut.dwfConcen"][p]
        q = lat
        pos = q > 0
        w = np.where(pos, q * dc, 0.0)
        w = np.where(pos, w + q * GRID_CONC[p], 0.0)
        w = np.where(pos, w - q * dc, 0.0)
        out[p] = w
    return out
