"""GPU vs the CPU restatement at sizes beyond the golden fixtures, plus
size-independent properties at the benchmark size.

* 100 x 100 grid (19,801 conduits) and a surcharged 60 x 60 variable-step
  grid: the engine's exported initial state seeds the oracle
  (oracle/dw_oracle.c, itself bit-identical to the reference), both run the
  same steps, state must agree within rtol 1e-6.
* 707 x 707 grid (998,285 conduits, the benchmark workload): bitwise
  run-to-run determinism (no atomics in any sum), finite state, and the
  flow-routing continuity error of the whole 5-minute run against the value
  the compiled reference reports for the same input
  (tests/golden/grid707_5min_reference.json; the reference's own figure is a
  large -18.7 % because the grid fills from dry).
"""
import json
import os

import numpy as np
import pytest

import netgen
import swmm5
from _dumpio import read_dump
from _oracle import oracle_from_dump

RTOL, ATOL = 1e-6, 1e-9


def _engine(inp, tmp_path, save=False):
    s = swmm5.SWMM()
    assert s.open(inp, str(tmp_path / "e.rpt"), str(tmp_path / "e.out")) == 0, s.getError()
    assert s.start(save) == 0, s.getError()
    return s


@pytest.mark.gpu
@pytest.mark.parametrize("nx,steps,kw", [
    (100, 60, dict(route_step=1.0)),
    (60, 80, dict(route_step=5.0, variable_step=0.75, diameter=1.0, q=0.1)),
    (40, 40, dict(route_step=2.0, pollutants=3)),
])
def test_gpu_matches_oracle(nx, steps, kw, tmp_path):
    inp = str(tmp_path / "g.inp")
    netgen.write_grid(inp, nx, nx, end_time="06:00:00", **kw)
    s = _engine(inp, tmp_path)
    dump = str(tmp_path / "init.bin")
    assert s.export_state(dump) == 0
    d = read_dump(dump)
    o = oracle_from_dump(d)
    q = kw.get("q", 0.02)
    lat = np.full(o.nN, q)
    lat[-1] = 0.0
    o.d("node.latIn")[:] = lat
    P = kw.get("pollutants", 0)
    if P:
        conc = [5.0, 10.0, 15.0]
        qi = o.d("node.qualIn").reshape(P, o.nN)
        for p in range(P):
            w = np.where(lat > 0, lat * conc[p], 0.0)
            w = np.where(lat > 0, w + lat * conc[p], 0.0)
            w = np.where(lat > 0, w - lat * conc[p], 0.0)
            qi[p] = w
    for k in range(steps):
        dt = o.routing_step(d["opt.d"][0])
        o.step(dt)
        err, _ = s.step()
        assert err == 0
    for f in ("newDepth", "newVolume", "inflow", "outflow"):
        np.testing.assert_allclose(s.get_array("node." + f), o.d("node." + f), rtol=RTOL, atol=ATOL,
                                   err_msg=f)
    for f in ("newFlow", "newDepth", "newVolume", "a1", "q1", "dqdh", "froude"):
        np.testing.assert_allclose(s.get_array("link." + f), o.d("link." + f), rtol=RTOL, atol=ATOL,
                                   err_msg=f)
    if P:
        np.testing.assert_allclose(s.get_array("node.newQual"), o.d("node.newQual"), rtol=RTOL,
                                   atol=ATOL)
        np.testing.assert_allclose(s.get_array("link.newQual"), o.d("link.newQual"), rtol=RTOL,
                                   atol=ATOL)
    c = s.counters()
    assert c["nonconverged"] == o.get("nonConverge")
    s.end()
    s.close()


@pytest.mark.gpu
def test_benchmark_grid_determinism_and_conservation(tmp_path):
    inp = "/tmp/swmm_bench_test_g707.inp"
    if not os.path.exists(inp):
        netgen.write_grid(inp, 707, 707, end_time="00:05:00", report_all=False)
    finals = []
    for rep in range(2):
        s = _engine(inp, tmp_path)
        err, t = s.run_steps(100)
        assert err == 0
        depth = s.get_array("node.newDepth")
        flow = s.get_array("link.newFlow")
        assert np.isfinite(depth).all() and np.isfinite(flow).all()
        assert (depth >= 0).all()
        c = s.counters()
        assert c["conduits"] == 998285 and c["steps"] == 100
        assert 2 <= c["iterations"] / c["steps"] <= 8
        finals.append((depth, flow))
        while True:
            err, t = s.step()
            assert err == 0
            if t == 0.0:
                break
        assert s.end() == 0
        _, ferr, _ = s.getMassBalErr()
        ref = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                          "grid707_5min_reference.json")))
        assert abs(ferr - ref["flow_routing_continuity"]["continuity_error_pct"]) < 0.002, ferr
        s.close()
    np.testing.assert_array_equal(finals[0][0], finals[1][0])
    np.testing.assert_array_equal(finals[0][1], finals[1][1])
