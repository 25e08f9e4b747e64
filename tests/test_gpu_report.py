"""Report file: the engine's summary tables against the reference's report.

For every golden case the engine runs to the end through the C ABI and its
report file (.rpt) is compared with the reference's report for the same
input (tests/golden/<case>.ref_rpt.txt, written by the compiled reference).
Each summary section (continuity, accuracy statistics, routing time-step
summary, node / outfall / link tables) must have the same lines; times of maxima
are not compared here (on a plateau of equal maxima a last-ulp difference picks
another step; test_gpu_stats checks those dates against the reference's own
series), numbers are compared to one unit in their last printed digit (a value whose rounding
boundary falls between the two builds' libm ulps may print one digit apart),
every other token must be identical.
"""
import os
import re

import pytest

import _golden
import swmm5

SECTIONS = ["Highest Continuity Errors", "Time-Step Critical Elements",
            "Highest Flow Instability Indexes", "Most Frequent Nonconverging Nodes",
            "Routing Time Step Summary", "Node Depth Summary", "Node Inflow Summary",
            "Node Surcharge Summary", "Node Flooding Summary", "Storage Volume Summary",
            "Outfall Loading Summary",
            "Link Flow Summary", "Flow Classification Summary", "Conduit Surcharge Summary",
            "Pumping Summary"]
NUM = re.compile(r"^[-+]?(\d+\.?\d*|\.\d+)(e[-+]?\d+)?%?$", re.I)


def _sections(text):
    lines = text.split("\n")
    out = {}
    stars = [i for i, l in enumerate(lines) if l.strip() and set(l.strip()) == {"*"}]
    for k, i in enumerate(stars[:-1]):
        if stars[k + 1] != i + 2:
            continue
        title = lines[i + 1].strip()
        end = next((s for s in stars[k + 2:] if s > i + 2), len(lines))
        body = [l.rstrip() for l in lines[i + 3:end]]
        while body and not body[-1].strip():
            body.pop()
        out[title] = body
    # continuity table: header line starts with stars then "Volume"
    for i, l in enumerate(lines):
        if l.strip().startswith("Flow Routing Continuity"):
            body = []
            for m in lines[i + 2:]:
                if not m.strip():
                    break
                body.append(m.rstrip())
            out["Flow Routing Continuity"] = body
    return out


TIME = re.compile(r"^(\d+):(\d\d)$")


def _tok_equal(a, b):
    if a == b:
        return True
    if TIME.match(a) and TIME.match(b):
        # time of a maximum: on a plateau of equal maxima a last-ulp difference
        # picks another step; test_gpu_stats checks every such date against
        # the reference's own series
        return True
    ta, tb = a.rstrip("%"), b.rstrip("%")
    if not (NUM.match(a) and NUM.match(b)):
        return False
    try:
        x, y = float(ta), float(tb)
    except ValueError:
        return False
    dec = max(len(ta.split(".")[1]) if "." in ta else 0, len(tb.split(".")[1]) if "." in tb else 0)
    return abs(x - y) <= 1.01 * 10.0 ** (-dec) + 1e-12 * max(abs(x), abs(y))


def _compare(mine, ref, title):
    assert len(mine) == len(ref), "%s: %d vs %d lines\n%s\n----\n%s" % (
        title, len(mine), len(ref), "\n".join(mine), "\n".join(ref))
    for a, b in zip(mine, ref):
        ta, tb = a.split(), b.split()
        ok = len(ta) == len(tb) and all(_tok_equal(x, y) for x, y in zip(ta, tb))
        assert ok, "%s:\n  mine: %s\n  ref : %s" % (title, a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("name", _golden.CASES)
def test_report_tables_match_reference(name, tmp_path):
    rpt, out = str(tmp_path / "r.rpt"), str(tmp_path / "r.out")
    s = swmm5.SWMM()
    assert s.open(_golden.inp(name), rpt, out) == 0, s.getError()
    assert s.start(True) == 0, s.getError()
    acts, done = _golden.actions(_golden.load(name)), 0
    while True:
        _golden.apply_actions(s, acts, done)
        err, t = s.step()
        done += 1
        assert err == 0, s.getError()
        if t == 0.0:
            break
    assert s.end() == 0
    s.report()
    s.close()
    mine = _sections(open(rpt, encoding="latin-1").read())
    ref = _sections(open(os.path.join(_golden.GOLDEN, name + ".ref_rpt.txt"), encoding="latin-1").read())
    checked = 0
    for title in ["Flow Routing Continuity"] + SECTIONS:
        if title not in ref:
            assert title not in mine, title
            continue
        assert title in mine, "missing section %s" % title
        _compare(mine[title], ref[title], title)
        checked += 1
    assert checked >= 10
