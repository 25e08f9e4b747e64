"""swmm_getValue / swmm_setValue during a run (swmm5.c:842-1213).

Between steps getValue reads the one value it needs straight from HBM (no
full state download); the values must equal the ones computed from the
synchronised host mirror bit for bit, and match the reference's state at
that step (rtol 1e-6, the north_star tolerance).  setValue's mid-run effects
(external inflow, outfall stage, routing step) are pinned by the
"example_api" golden case in test_gpu_parity / test_oracle_vs_reference.
"""
import numpy as np
import pytest

import _golden
import swmm5

NODE_PROPS = [swmm5.NODE_DEPTH, swmm5.NODE_HEAD, swmm5.NODE_VOLUME, swmm5.NODE_LATFLOW,
              swmm5.NODE_INFLOW, swmm5.NODE_OVERFLOW]
LINK_PROPS = [swmm5.LINK_FLOW, swmm5.LINK_DEPTH, swmm5.LINK_VELOCITY, swmm5.LINK_TOPWIDTH,
              swmm5.LINK_SETTING]


@pytest.mark.gpu
def test_getvalue_from_device_equals_mirror_and_reference(tmp_path):
    name = "example_api"
    d = _golden.load(name)
    acts = _golden.actions(d)
    s = swmm5.SWMM()
    assert s.open(_golden.inp(name), str(tmp_path / "a.rpt"), str(tmp_path / "a.out")) == 0
    assert s.start(False) == 0, s.getError()
    nn, nl = s.getCount(swmm5.NODE), s.getCount(swmm5.LINK)
    checked = 0
    for step in range(1, 301):
        err, t = _golden.advance(s, acts, step - 1)
        assert err == 0, s.getError()
        if step % 37:
            continue
        dev_n = [[s.getValue(p, i) for i in range(nn)] for p in NODE_PROPS]
        dev_l = [[s.getValue(p, j) for j in range(nl)] for p in LINK_PROPS]
        depth = s.get_array("node.newDepth")            # synchronises the mirror
        host_n = [[s.getValue(p, i) for i in range(nn)] for p in NODE_PROPS]
        host_l = [[s.getValue(p, j) for j in range(nl)] for p in LINK_PROPS]
        np.testing.assert_array_equal(np.array(dev_n), np.array(host_n))
        np.testing.assert_array_equal(np.array(dev_l), np.array(host_l))
        np.testing.assert_allclose(depth, d["s.node.newDepth"][step - 1], rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(np.array(dev_n[0]), d["s.node.newDepth"][step - 1],
                                   rtol=1e-6, atol=1e-9)
        checked += 1
    assert checked >= 8
    s.end()
    s.close()


@pytest.mark.gpu
def test_setvalue_routestep_switches_to_fixed_steps(tmp_path):
    s = swmm5.SWMM()
    assert s.open(_golden.inp("example_var"), str(tmp_path / "b.rpt"), str(tmp_path / "b.out")) == 0
    assert s.start(False) == 0, s.getError()
    for _ in range(20):
        assert s.step()[0] == 0
    s.setValue(swmm5.ROUTESTEP, -1, 2.5)
    assert s.getValue(swmm5.ROUTESTEP, -1) == 2.5
    t0 = s.getValue(swmm5.ELAPSEDTIME, -1)
    for _ in range(4):
        assert s.step()[0] == 0
    t1 = s.getValue(swmm5.ELAPSEDTIME, -1)
    assert abs((t1 - t0) * 86400.0 - 10.0) < 1e-6
    s.end()
    s.close()
