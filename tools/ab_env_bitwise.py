"""A/B bitwise check of one environment switch: the 60 x 60 surcharged
variable-step grid, 300 steps, run with VAR=A and VAR=B (plus any fixed
KEY=VALUE pairs), every node and link state array and the iteration counts
compared.  usage: ab_env_bitwise.py VAR A B [KEY=VALUE ...]"""
import os, sys, tempfile
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "stormwater-management-model_amd"))
import netgen, swmm5
var, va, vb = sys.argv[1:4]
for kv in sys.argv[4:]:
    k, v = kv.split("=", 1)
    os.environ[k] = v
d = tempfile.mkdtemp()
inp = os.path.join(d, "g.inp")
netgen.write_grid(inp, 60, 60, end_time="02:00:00", route_step=5.0, variable_step=0.75, diameter=1.0, q=0.3)
F = ["node." + f for f in ("newDepth", "newVolume", "inflow", "outflow", "overflow")] + \
    ["link." + f for f in ("newFlow", "newDepth", "newVolume", "a1", "q1", "dqdh", "froude")]
res = []
for val in (va, vb):
    os.environ[var] = val
    s = swmm5.SWMM()
    assert s.open(inp, os.path.join(d, "a.rpt"), os.path.join(d, "a.out")) == 0
    assert s.start(False) == 0
    snaps = []
    for _ in range(6):
        assert s.run_steps(50)[0] == 0, s.getError()
        snaps.append([s.get_array(n) for n in F])
    res.append((snaps, s.counters()))
    s.end(); s.close()
for a, b in zip(res[0][0], res[1][0]):
    for n, x, y in zip(F, a, b):
        assert np.array_equal(x, y), n
for k in ("steps", "iterations", "nonconverged"):
    assert res[0][1][k] == res[1][1][k], k
print("%s=%s vs %s bitwise ok:" % (var, va, vb), {k: res[1][1][k] for k in ("steps", "iterations", "steps_list")})
