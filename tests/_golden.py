"""Golden-fixture helpers (test infrastructure only)."""
from __future__ import annotations

import os
import shutil
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
CASES = ["grid12", "grid12_var_qual", "grid10_surcharge", "example", "example_var",
         "example_qual", "example_hotsave", "example_hot", "example_api", "example_storage",
         "example_storage_var", "example_storage_qual", "example_regulators",
         "example_regulators_var_qual", "example_shapes", "example_shapes_var",
         "example_irregular", "example_irregular_var", "example_culverts", "example_culverts_var",
         "example_tidal", "example_tidal_var", "example_roadway", "example_dividers",
         "example_streets", "example_extfile", "example_branches", "example_branches_var",
         "example_slot_pond", "example_options", "grid10_slot", "example_stride",
         "example_stride_fixed", "example_dummy", "example_dummy_var", "example_evap_monthly",
         "example_evap_series", "example_avg", "example_exfil", "example_exfil_var",
         "example_evap_file", "example_evap_temp", "example_evap_td3200", "example_evap_dly",
         "example_steady", "example_steady_var", "example_steady_pump"]
# cases using objects outside the C restatement's scope (oracle/dw_oracle.c
# covers junctions, outfalls and conduits): pinned by the GPU tests against the
# reference's own fixtures only
BEYOND_ORACLE = {"example_storage", "example_storage_var", "example_storage_qual",
                 "example_regulators", "example_regulators_var_qual", "example_shapes",
                 "example_shapes_var", "example_irregular", "example_irregular_var",
                 "example_culverts", "example_culverts_var", "example_tidal", "example_tidal_var",
                 "example_roadway", "example_dividers", "example_streets", "example_branches",
                 "example_branches_var", "example_dummy", "example_dummy_var",
                 "example_evap_monthly", "example_evap_series", "example_avg", "example_exfil",
                 "example_exfil_var", "example_evap_file", "example_evap_temp", "example_evap_td3200",
                 "example_evap_dly",
                 # swmm_stride calls: an API driver the C restatement does not model
                 "example_stride", "example_stride_fixed",
                 # SKIP_STEADY_STATE: routing_execute's steady-state skip (routing.c:383-395)
                 # is not in the restatement's step
                 "example_steady", "example_steady_var", "example_steady_pump"}
# cases whose input writes a file next to itself ([FILES] SAVE ...): they run
# from a private copy so the fixtures directory is never written to
SAVES = {"example_hotsave": "example_hotsave.hsf"}
# DWF-only networks: lateral inflow is constant and pollutant loads are
# q * concentration, so the oracle can be fed without the inflow machinery
DWF_ONLY = {"grid12", "grid12_var_qual", "grid10_surcharge", "grid10_slot"}
GRID_CONC = [5.0, 10.0, 15.0, 20.0, 25.0, 30.0]


# ill-conditioned cases: the fixture carries the reference's build-to-build
# spread ("env.*", tests/golden/make_golden.py ENVELOPE)
ENVELOPE = {"example_shapes", "example_shapes_var", "example_irregular", "example_irregular_var",
            "example_culverts", "example_culverts_var", "example_streets", "example_branches",
            "example_branches_var", "example_dummy", "example_dummy_var"}


def first_divergence(d, node_f, link_f, rtol, atol):
    """First recorded step index at which the reference's two builds (plain
    and FMA) differ by more than the tolerance in any checked state array."""
    n = len(d["env.node.newDepth"])
    first = n
    for pre, fs in (("node.", node_f), ("link.", link_f)):
        for f in fs:
            e, ref = d["env." + pre + f], d["s." + pre + f]
            bad = np.nonzero(e > atol + rtol * np.abs(ref).max(axis=1))[0]
            if bad.size:
                first = min(first, int(bad[0]))
    return first


def load(name: str) -> dict:
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def inp(name: str) -> str:
    src = os.path.join(GOLDEN, name + ".inp")
    if name not in SAVES:
        return src
    d = tempfile.mkdtemp(prefix="swmm_golden_")
    shutil.copy(src, d)
    return os.path.join(d, name + ".inp")


def ref_out(name: str) -> bytes:
    return np.load(os.path.join(GOLDEN, name + ".ref_out.npy"), allow_pickle=False).tobytes()


def fma_out(name: str) -> bytes:
    """The reference FMA build's binary results (ill-conditioned cases)."""
    return np.load(os.path.join(GOLDEN, name + ".fma_out.npy"), allow_pickle=False).tobytes()


def fma_rpt(name: str) -> str:
    with open(os.path.join(GOLDEN, name + ".fma_rpt.txt")) as f:
        return f.read()


def x87_rpt(name: str) -> str | None:
    """The reference x87 build's report (ill-conditioned cases), if stored."""
    p = os.path.join(GOLDEN, name + ".x87_rpt.txt")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return f.read()


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


# ------------------------------------------------------------------ API cases
# swmm_setValue calls the reference run made between steps (make_golden.py
# ACTIONS, recorded as "api.actions"): (afterStep, property, objectName, value)
def actions(d: dict) -> list:
    if "api.actions" not in d:
        return []
    out = []
    for tok in bytes(d["api.actions"]).decode().split(";"):
        at, prop, name, val = tok.split(":")
        out.append((int(at), int(prop), name, float(val)))
    return out


def apply_actions(s, acts: list, done: int) -> int:
    """Make the same swmm_setValue calls on engine `s` once `done` steps ran;
    returns the seconds of a swmm_stride that replaces the next swmm_step
    (property -1 in the fixture), else 0."""
    stride = 0
    for at, prop, name, val in acts:
        if at != done:
            continue
        if prop == -1:
            stride = int(val)
            continue
        idx = -1
        if name != "-":
            idx = s.getIndex(2 if prop < 400 else 3, name)
            assert idx >= 0, name
        s.setValue(prop, idx, val)
    return stride


def advance(s, acts: list, done: int):
    """The reference run's next call after `done` calls: its setValue calls,
    then swmm_step or swmm_stride; returns (error, elapsed days)."""
    stride = apply_actions(s, acts, done)
    return s.stride(stride) if stride > 0 else s.step()
