#!/usr/bin/env python3
"""Per-step kernel sequence from a rocprofv3 --kernel-trace CSV: duration of
every dispatch of the last N routing steps (a step ends at k_finalize) and the
mean per kernel class and iteration position.

usage: step_trace.py <kernel_trace.csv> [N]"""
import collections
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 re.sub(r"\(swx::Params.*", "", r["Kernel_Name"]).replace("void swx::", ""))
                for r in rows)
    steps, cur = [], []
    for e in ev:
        if e[2].startswith("__amd"):
            continue
        cur.append(e)
        if e[2].startswith("k_finalize"):
            steps.append(cur)
            cur = []
    steps = steps[-n - 5:-5]         # the timed window, not the timing launches after it
    pos = collections.defaultdict(list)
    spans = []
    for s in steps:
        spans.append((s[-1][1] - s[0][0]) / 1e3)
        seen = collections.Counter()
        for e in s:
            seen[e[2]] += 1
            pos[(e[2], seen[e[2]])].append((e[1] - e[0]) / 1e3)
    print("steps %d  mean span %.1f us" % (len(steps), sum(spans) / len(spans)))
    tot = 0.0
    for (k, i), v in sorted(pos.items(), key=lambda kv: min(kv[1])):
        pass
    for (k, i), v in sorted(pos.items()):
        m = sum(v) / len(steps)
        tot += m
        print("  %-40s #%d  %6.1f us/step  (%d steps)" % (k[:40], i, m, len(v)))
    print("  kernel total %.1f us/step" % tot)


if __name__ == "__main__":
    main()
