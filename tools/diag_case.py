"""Diagnostic: per-step relative deviation of the engine from a golden case
(test infrastructure; prints the first steps where any node/link state
deviates by more than a threshold, with the object ids)."""
import sys
import os
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "stormwater-management-model_amd"))
import _golden  # noqa: E402
import swmm5  # noqa: E402

name = sys.argv[1]
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-9
d = _golden.load(name)
s = swmm5.SWMM()
assert s.open(_golden.inp(name), "/tmp/diag.rpt", "/tmp/diag.out") == 0
assert s.start(False) == 0
acts = _golden.actions(d)
nl = s.getCount(swmm5.LINK)
nn = s.getCount(swmm5.NODE)
lid = [s.getName(swmm5.LINK, j) for j in range(nl)]
nid = [s.getName(swmm5.NODE, j) for j in range(nn)]
total = int(d["s.every"][1])
shown = 0
for step in range(1, total + 1):
    _golden.apply_actions(s, acts, step - 1)
    s.step()
    rec = step - 1
    out = []
    for f, ids, pre in (("newFlow", lid, "link."), ("newDepth", lid, "link."), ("newDepth", nid, "node."),
                        ("inflow", nid, "node.")):
        a = s.get_array(pre + f)
        b = d["s." + pre + f][rec]
        r = np.abs(a - b) / (np.abs(b) + 1e-12)
        k = int(np.argmax(r))
        if r[k] > thr:
            out.append("%s%s[%s] %.3e (%.9g vs %.9g)" % (pre, f, ids[k], r[k], a[k], b[k]))
    if out:
        print("step", step, "dt", d["s.dt"][rec], "; ".join(out))
        shown += 1
        if shown > 40:
            break
