"""A/B bitwise check of two engine builds on the surcharged grids
(diagnostic): runs the 60 x 60 grid (q = 0.3, 300 steps) and the benchmark's
707 x 707 grid (q = 0.12, 800 steps, into the surcharged regime) with each
library and compares every node and link state array and the counters.
  python tools/ab_grid.py <libA.so> <libB.so>"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stormwater-management-model_amd"))
sys.path.insert(0, ROOT)
import netgen  # noqa: E402
import swmm5   # noqa: E402

F = ["node." + f for f in ("newDepth", "newVolume", "inflow", "outflow", "overflow")] + \
    ["link." + f for f in ("newFlow", "newDepth", "newVolume", "a1", "q1", "dqdh", "froude", "surfArea1",
                           "surfArea2")]


def run(lib, inp, steps, d):
    s = swmm5.SWMM(lib)
    assert s.open(inp, os.path.join(d, "a.rpt"), os.path.join(d, "a.out")) == 0, s.getError()
    assert s.start(False) == 0, s.getError()
    snaps = []
    done = 0
    while done < steps:
        n = min(100, steps - done)
        assert s.run_steps(n)[0] == 0, s.getError()
        done += n
        snaps.append([s.get_array(f) for f in F])
    c = s.counters()
    s.end()
    s.close()
    return snaps, c


def main():
    a, b = sys.argv[1], sys.argv[2]
    d = tempfile.mkdtemp()
    cases = []
    g60 = os.path.join(d, "g60.inp")
    netgen.write_grid(g60, 60, 60, end_time="02:00:00", route_step=5.0, variable_step=0.75, diameter=1.0, q=0.3)
    cases.append(("60x60", g60, 300))
    import bench
    cfg = bench.PRESETS["1m_surcharge"]
    cases.append(("707x707", bench.make_inp(cfg["grid"], cfg["route_step"], cfg["variable_step"], cfg["pollutants"],
                                            cfg["diameter"], cfg["q"]), 800))
    for name, inp, steps in cases:
        ra, rb = run(a, inp, steps, d), run(b, inp, steps, d)
        for sa, sb in zip(ra[0], rb[0]):
            for f, x, y in zip(F, sa, sb):
                assert np.array_equal(x, y), (name, f, float(np.max(np.abs(x - y))))
        for k in ("steps", "iterations", "nonconverged"):
            assert ra[1][k] == rb[1][k], (name, k, ra[1][k], rb[1][k])
        print(name, "bitwise equal:", {k: ra[1][k] for k in ("steps", "iterations", "nonconverged")})


if __name__ == "__main__":
    main()
