"""Pins the CPU restatement (oracle/dw_oracle.c) to the reference solver.

Replays every golden case -- state dumps of the compiled reference
(oracle/refdump.c, captured by tests/golden/make_golden.py) -- through the
restatement, starting from the reference's own post-swmm_start state, and
requires BIT-IDENTICAL node and link state after every recorded routing step,
plus identical variable time steps.  This is what makes the oracle a valid
checker for the MI355X path.
"""
import numpy as np
import pytest

import _golden
import swmm5
from _oracle import oracle_from_dump

NODE_F = ["newDepth", "newVolume", "inflow", "outflow", "overflow"]
LINK_F = ["newFlow", "newDepth", "newVolume", "froude", "dqdh", "surfArea1", "surfArea2", "a1",
          "q1"]
LINK_I = ["flowClass", "fullState", "capacityLimited", "normalFlow"]


def _replay(name):
    d = _golden.load(name)
    o = oracle_from_dump(d)
    ev = _golden.every(d)
    nrec = len(d["s.dt"])
    nn, nl, P = (int(x) for x in d["counts"][:3])
    total = int(d["s.every"][1])
    dwf = name in _golden.DWF_ONLY
    rec = 0
    fixed = d["opt.d"][0]
    acts = _golden.actions(d)
    ids = {}
    if acts:                                   # object names -> indices (host-only open)
        s = swmm5.SWMM()
        assert s.open(_golden.inp(name), "/tmp/_orc_api.rpt", "/tmp/_orc_api.out") == 0
        for _, prop, nm, _ in acts:
            if nm != "-":
                ids[nm] = s.getIndex(swmm5.NODE if prop < 400 else swmm5.LINK, nm)
        s.close()
    for step in range(1, total + 1):
        for at, prop, nm, val in acts:         # swmm_setValue between steps
            if at != step - 1:
                continue
            if prop == swmm5.ROUTESTEP:        # setRoutingStep (swmm5.c:1360-1370)
                o.opt("courantFactor", 0.0)
                fixed = max(val, o.get("minRouteStep"))
            elif prop == swmm5.NODE_HEAD:      # setOutfallStage (swmm5.c:1173-1188), CFS units
                o.d("node.fixedStage")[ids[nm]] = val
                o.i("node.outfallType")[ids[nm]] = 2
        dt = o.routing_step(fixed)
        if dwf:
            lat = d["s.node.newLatFlow"][0]
        else:
            assert ev == 1
            lat = d["s.node.newLatFlow"][step - 1]
        o.d("node.latIn")[:] = lat
        if P and dwf:
            o.d("node.qualIn")[:] = _golden.grid_qual_loads(d, lat).ravel()
        if step % ev == 0 or step == total:
            dt_ref = d["s.dt"][rec]
            if step < total:
                assert dt == dt_ref, (name, step, dt, dt_ref)
            dt = dt_ref
        o.step(dt)
        if step % ev == 0 or step == total:
            for f in NODE_F:
                np.testing.assert_array_equal(o.d("node." + f), d["s.node." + f][rec],
                                              err_msg="%s step %d node.%s" % (name, step, f))
            for f in LINK_F:
                np.testing.assert_array_equal(o.d("link." + f), d["s.link." + f][rec],
                                              err_msg="%s step %d link.%s" % (name, step, f))
            for f in LINK_I:
                np.testing.assert_array_equal(o.i("link." + f), d["s.link." + f][rec],
                                              err_msg="%s step %d link.%s" % (name, step, f))
            if P and dwf:
                for p in range(P):
                    np.testing.assert_array_equal(
                        o.d("node.newQual").reshape(P, nn)[p], d["s.node.qual%d" % p][rec])
                    np.testing.assert_array_equal(
                        o.d("link.newQual").reshape(P, nl)[p], d["s.link.qual%d" % p][rec])
            rec += 1
    assert rec == nrec
    assert o.get("nonConverge") == d["run.counts"][0]
    return d


@pytest.mark.parametrize("name", [c for c in _golden.CASES if c not in _golden.BEYOND_ORACLE])
def test_oracle_bit_identical_to_reference(name):
    _replay(name)


def test_surcharge_case_exercises_surcharge_and_nonconvergence():
    d = _golden.load("grid10_surcharge")
    assert d["run.counts"][0] > 0            # some steps hit MaxTrials
    depth = d["s.node.newDepth"]
    crown = d["node.crownElev"] - d["node.invertElev"]
    assert (depth > crown[None, :]).any()    # EXTRAN surcharge branch taken


def test_example_exercises_flow_classes():
    d = _golden.load("example")
    fc = np.bincount(d["s.link.flowClass"].ravel(), minlength=7)
    assert fc[0] > 0 and fc[1] > 0 and fc[3] > 0 and fc[4] > 0 and fc[6] > 0
