"""The bench's default multi-GPU partition, checked on the CPU: the two-region
partition (swmmx_setPartitionMode(1)) that bench.py --balance auto builds
from profiles/partition_weights.json (tools/calibrate_partition.py's per-row
sparse work, measured on one GPU) must share that measured work and the node
count evenly between the ranks, for the weak-scaling grid two ranks run.
The layout is the engine's own (swmmx_getOwner after swmm_open, no GPU); the
per-rank work is the record's rows summed over each rank's nodes.  The GPU
rehearsals measure the same thing live (profiles/r06_rehearsal_*.json,
DESIGN.md section 6)."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "stormwater-management-model_amd"))

import swmm5  # noqa: E402

RECORDS = os.path.join(ROOT, "profiles", "partition_weights.json")


def _records():
    return json.load(open(RECORDS)) if os.path.exists(RECORDS) else {}


def test_records_are_well_formed():
    recs = _records()
    assert recs, "profiles/partition_weights.json holds no calibration record"
    for key, r in recs.items():
        rows, nx = r["rows"], r["nx"]
        assert r["nodes"] == rows * nx + 1, key                  # the grid and its outfall
        assert len(r["row_updates"]) == rows and len(r["row_conduit_updates"]) == rows, key
        assert min(r["row_updates"]) >= 0.0 and min(r["row_conduit_updates"]) >= 0.0, key
        s = r["sparse_us"]
        assert s["reliable"] and s["b_per_update"] > 0.0 and r["lambda"] > 0.0, key
        assert r["backend"].startswith("hip:gfx950"), key


@pytest.mark.parametrize("world", [2])
def test_two_region_partition_balances_the_measured_work(world, tmp_path):
    import bench
    cfg = dict(bench.PRESETS["1m_surcharge"])
    rows, nx = cfg["grid"] * world, cfg["grid"]
    key = bench.workload_name("1m_surcharge", cfg, rows)
    rec = _records().get(key)
    if rec is None:
        pytest.skip("no calibration record for " + key)
    n_nodes = rows * nx + 1
    w, rec = bench.partition_weights(key, rows, nx, n_nodes)
    assert w is not None
    inp = bench.make_inp(nx, cfg["route_step"], cfg["variable_step"], cfg["pollutants"], cfg["diameter"],
                         cfg["q"], rows=rows)
    s = swmm5.SWMM()
    s.set_partition(0, world)
    s.set_partition_weights(w)
    assert s.set_partition_mode("two_region") == 0
    try:
        assert s.open(inp, str(tmp_path / "p.rpt"), str(tmp_path / "p.out")) == 0, s.getError()
        owner = s.owners(swmm5.NODE)
    finally:
        s.close()
        s.set_partition_mode("contiguous")
        s.set_partition_weights(None)
        s.set_partition(0, 1)
    grid = owner[:rows * nx]
    un = np.repeat(np.asarray(rec["row_updates"]) / nx, nx)
    uc = np.repeat(np.asarray(rec["row_conduit_updates"]) / nx, nx)
    nodes = np.bincount(grid, minlength=world)
    node_work = np.bincount(grid, weights=un, minlength=world)
    conduit_work = np.bincount(grid, weights=uc, minlength=world)
    # row strips for comparison: the band sits in the last strip
    strips = np.arange(rows * nx) * world // (rows * nx)
    strip_work = np.bincount(strips, weights=un, minlength=world)
    assert strip_work.max() / strip_work.min() > 1.5, strip_work
    assert nodes.max() / nodes.min() < 1.05, nodes
    assert node_work.max() / node_work.min() < 1.3, node_work
    assert conduit_work.max() / conduit_work.min() < 1.3, conduit_work
