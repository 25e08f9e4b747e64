"""bench.py's use of the committed profile records (CPU only): the in-graph
k_link<first> duration (profiles/kernel_timing.json) and the PMC bytes
(profiles/pmc_traffic.json) are taken only for the same workload, device,
engine sources (sha256 of every source, header and the Makefile) and regime
(same spin-up: any warm-up / step count, so the driver's --steps 20
--warmup 5 invocation matches a profile of that window); every record is
well formed and names a summary that exists under profiles/."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROFILES = os.path.join(ROOT, "profiles")


def test_same_regime_rule():
    assert bench.same_regime(None, [750, 5, 20])
    assert bench.same_regime([750, 5, 20], [750, 5, 20])
    assert bench.same_regime([750, 20, 200], [750, 5, 20])          # another window, same spin-up
    assert not bench.same_regime([400, 20, 200], [750, 5, 20])      # another regime
    assert not bench.same_regime([750, 5], [750, 5, 20])


def _records(name):
    with open(os.path.join(PROFILES, name)) as f:
        return json.load(f)


def test_records_are_well_formed():
    for name, keys in (("kernel_timing.json", ("kernel", "avg_launch_us", "launches", "window", "src_sha",
                                               "backend", "source")),
                       ("pmc_traffic.json", ("bytes_per_launch", "step_bytes", "iterations_per_step", "window",
                                             "calibration", "src_sha", "backend", "source"))):
        recs = _records(name)
        assert recs, name
        for workload, rec in recs.items():
            for k in keys:
                assert k in rec, (name, workload, k)
            assert len(rec["window"]) == 3, (name, workload)
            assert rec["backend"].startswith("hip:gfx950"), (name, workload)
            summary = rec["source"].split()[0]
            assert os.path.exists(os.path.join(ROOT, summary)), (name, workload, summary)
            # a record names a preset's workload (the bench builds the same string)
            assert workload.split(":")[0] in bench.PRESETS, workload


def test_records_matched_only_for_their_source_and_device(monkeypatch):
    import swmm5
    recs = _records("kernel_timing.json")
    workload, rec = next(iter(recs.items()))
    backend = rec["backend"]
    monkeypatch.setattr(swmm5, "kernel_source_sha", lambda: rec["src_sha"])
    assert bench.timing_record(workload, rec["window"], backend) == rec
    assert bench.timing_record(workload, [rec["window"][0], 5, 20], backend) == rec
    assert bench.timing_record(workload, [rec["window"][0] + 1, 5, 20], backend) is None
    assert bench.timing_record(workload, rec["window"], "hip:gfx942") is None
    monkeypatch.setattr(swmm5, "kernel_source_sha", lambda: "0" * 16)
    assert bench.timing_record(workload, rec["window"], backend) is None
