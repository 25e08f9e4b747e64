#!/usr/bin/env python3
"""Per-position averages of rocprofv3 --pmc counters within a routing step
(a step starts at k_link<true ...>), over the last N steps.
usage: pmc_positions.py <run_counter_collection.csv> [last_n_steps]"""
import collections
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    disp = collections.OrderedDict()
    for r in rows:
        d = int(r["Dispatch_Id"])
        name = re.sub(r"\(swx::Params.*", "", r["Kernel_Name"]).replace("void swx::", "")
        disp.setdefault(d, [name, {}])
        disp[d][1][r["Counter_Name"]] = disp[d][1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    steps, cur = [], []
    for d in sorted(disp):
        name, c = disp[d]
        if name.startswith("k_link<true"):
            if cur:
                steps.append(cur)
            cur = []
        cur.append((name, c))
    if cur:
        steps.append(cur)
    steps = [s for s in steps if len(s) >= 4][-last:]
    npos = max(len(s) for s in steps)
    names = sorted({k for s in steps for _, c in s for k in c})
    print("pos kernel " + " ".join(names))
    for i in range(npos):
        acc = collections.defaultdict(float)
        n = 0
        kn = ""
        for s in steps:
            if i < len(s):
                kn = s[i][0]
                n += 1
                for k, v in s[i][1].items():
                    acc[k] += v
        print("%2d %-28s %s" % (i, kn[:28], " ".join("%.4g" % (acc[k] / max(n, 1)) for k in names)))


if __name__ == "__main__":
    main()
