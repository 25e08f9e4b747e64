#!/usr/bin/env python3
"""Average duration of each kernel position within a routing step, from a
rocprofv3 --kernel-trace CSV (a step starts at k_link<true ...>).

usage: step_positions.py <kernel_trace.csv> [last_n_steps]"""
import collections
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 re.sub(r"\(swx::Params.*", "", r["Kernel_Name"]).replace("void swx::", ""))
                for r in rows)
    steps, cur = [], []
    for e in ev:
        if e[2].startswith("k_link<true"):
            if cur:
                steps.append(cur)
            cur = []
        cur.append(e)
    steps.append(cur)
    sel = [s for s in steps if any(x[2].startswith("k_finalize") for x in s)
           and not any(x[2].startswith("__amd") for x in s)]
    sel = sel[-last:]
    pos = collections.defaultdict(list)
    for s in sel:
        for i, e in enumerate(s):
            pos[(i, e[2][:26])].append(e[1] - e[0])
        pos[(99, "step (first start .. last end)")].append(s[-1][1] - s[0][0])
    tot = 0.0
    for k, v in sorted(pos.items()):
        us = sum(v) / len(v) / 1000
        if k[0] != 99:
            tot += us
        print("%3d %-32s %4d %8.2f us" % (k[0], k[1], len(v), us))
    print("    kernels total %.2f us" % tot)


if __name__ == "__main__":
    main()
