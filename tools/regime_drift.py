#!/usr/bin/env python3
"""Diagnostic (GPU box): engine vs oracle drift in the surcharged regime.

Runs the 100 x 100 surcharge case in lockstep from the start and prints, every
10 steps, the largest relative difference of node depth and link flow
(|a - b| / max(|b|, 1e-3)), the iteration counts, and the same figures for a
window restarted from the engine's own state (oracle_resume) at given steps."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "stormwater-management-model_amd"), os.path.join(ROOT, "tests"), ROOT):
    sys.path.insert(0, p)
import netgen  # noqa: E402
import swmm5  # noqa: E402
from _dumpio import read_dump  # noqa: E402
from _oracle import oracle_from_dump, oracle_resume  # noqa: E402


def rel(a, b):
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-3)))


def main():
    nx = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    q = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
    tmp = "/tmp/drift"
    os.makedirs(tmp, exist_ok=True)
    inp = os.path.join(tmp, "g.inp")
    netgen.write_grid(inp, nx, nx, end_time="01:00:00", route_step=5.0, variable_step=0.75,
                      diameter=1.0, q=q)
    s = swmm5.SWMM()
    assert s.open(inp, tmp + "/e.rpt", tmp + "/e.out") == 0
    assert s.start(False) == 0
    s.export_state(tmp + "/init.bin")
    d = read_dump(tmp + "/init.bin")
    o = oracle_from_dump(d)
    lat = np.full(o.nN, q)
    lat[-1] = 0
    o.d("node.latIn")[:] = lat
    win = None
    k = 0
    while True:
        dt = o.routing_step(5.0)
        it = o.step(dt)
        if win is not None:
            win.step(win.routing_step(5.0))
        err, t = s.step()
        k += 1
        c = s.counters()
        if k % 10 == 0 or c["last_iterations"] != it or (win is not None and k % 10 < 5):
            dep, fl = s.get_array("node.newDepth"), s.get_array("link.newFlow")
            line = "step %4d it gpu %d orc %d  nonconv gpu %d orc %d  depth %.2e flow %.2e" % (
                k, c["last_iterations"], it, c["nonconverged"], o.get("nonConverge"),
                rel(dep, o.d("node.newDepth")), rel(fl, o.d("link.newFlow")))
            if win is not None:
                line += "  | window depth %.2e flow %.2e" % (rel(dep, win.d("node.newDepth")),
                                                            rel(fl, win.d("link.newFlow")))
            print(line, flush=True)
        if k in (300, 450, 550, 650):
            s.export_state(tmp + "/mid.bin")
            win = oracle_resume(read_dump(tmp + "/mid.bin"))
            win.d("node.latIn")[:] = lat
        if t == 0.0 or err:
            break


if __name__ == "__main__":
    main()
