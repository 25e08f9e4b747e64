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
    for step in range(1, total + 1):
        dt = o.routing_step(d["opt.d"][0])
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


@pytest.mark.parametrize("name", _golden.CASES)
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
