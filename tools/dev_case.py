"""Diagnostic: per-step largest |engine - reference| of every recorded state
array of a golden case, saved to gpurun_out/dev_<case>.npz (with the counters)
for offline comparison with the reference's own build-to-build envelope."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "stormwater-management-model_amd"))
import _golden  # noqa: E402
import swmm5  # noqa: E402

name = sys.argv[1]
d = _golden.load(name)
s = swmm5.SWMM()
assert s.open(_golden.inp(name), "/tmp/dev.rpt", "/tmp/dev.out") == 0
assert s.start(False) == 0
acts = _golden.actions(d)
ev = _golden.every(d)
total = int(d["s.every"][1])
keys = [k[2:] for k in d if k.startswith("s.node.") or k.startswith("s.link.")]
keys = [k for k in keys if d["s." + k].dtype == np.float64 and "qual" not in k]
dev = {k: [] for k in keys}
arg = {k: [] for k in keys}
fcls = []
rec = 0
for step in range(1, total + 1):
    _golden.apply_actions(s, acts, step - 1)
    s.step()
    if step % ev == 0 or step == total:
        for k in keys:
            try:
                a = s.get_array(k)
            except Exception:
                continue
            b = d["s." + k][rec]
            if a.shape == b.shape:
                dev[k].append(np.abs(a - b).max())
                arg[k].append(int(np.argmax(np.abs(a - b))))
        fcls.append(s.get_array("link.flowClass"))
        rec += 1
s.step()
c = s.counters()
s.end()
_, ferr, _ = s.getMassBalErr()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "dev_%s.npz" % name),
         **{"dev." + k: np.array(v) for k, v in dev.items() if v},
         **{"arg." + k: np.array(v) for k, v in arg.items() if v}, fclass=np.array(fcls),
         nonconverged=c["nonconverged"], ferr=ferr)
print(name, "nonconverged", c["nonconverged"], "ref", d["run.counts"][0], "flow err", ferr, d["run.massbal"][1])
