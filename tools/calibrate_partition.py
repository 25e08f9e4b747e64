#!/usr/bin/env python3
"""Partition weights for bench.py's multi-GPU runs, measured on one GPU.

The sparse Picard iterations (k >= 2) follow the surcharge, which builds up
next to the outlet: contiguous row strips of equal size leave the strip
holding the outlet with several times the others' sparse work (DESIGN.md
section 6).  This tool runs a bench workload's whole grid on one GPU through
its spin-up, then times --steps steps (timing mode) and records

  * per grid row, the node updates per step in iterations k >= 2
    (swmmx_getNodeWork: the measured sparse work, node by node);
  * the cost of a rank's work that follows its node count (per node and
    step: the full passes of iterations 0 and 1 and the step end) and the
    marginal cost b of one sparse node update.  A sparse iteration k >= 3
    (list walk + node-list update, both driven by the live list, not by the
    grid) takes t = f + b u per launch pair for u live node updates, f the
    launch floor every rank pays alike.  Within one window u hardly changes
    from one iteration to the next (and k = 2 also rebuilds the lists), so b
    comes from two windows of the same run at different surcharge depths:
    window A --early-frac of the way through the spin-up, window B at the
    bench window itself, b = (t_B - t_A) / (u_B - u_A) over their mean
    k >= 3 iterations, f = t_B - b u_B.  The node weights use window B's
    per-node work.

bench.py --balance (the default with several ranks) then weighs node i of
row r as 1 + (b / c_node) * u_r / nx, and swmmx_setPartitionWeights cuts the
node order into contiguous blocks of equal weight.  Results go to
profiles/partition_weights.json under bench.py's workload name.

    python tools/calibrate_partition.py --config 4m
    python tools/calibrate_partition.py --config 1m_surcharge --gpus 8   # the weak-scaling grid of 8 ranks
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "stormwater-management-model_amd"))

os.environ.setdefault("SWMM5_SPARSE", "3")   # the list graph, as every rank of a partitioned run
import bench  # noqa: E402
import swmm5  # noqa: E402

OUT = os.path.join(ROOT, "profiles", "partition_weights.json")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4m", choices=sorted(bench.PRESETS))
    ap.add_argument("--gpus", type=int, default=2, help="rank count whose grid (weak scaling) and spin-up apply")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--early-frac", type=float, default=0.7,
                    help="window A starts at this fraction of the spin-up (a shallower surcharge)")
    args = ap.parse_args()
    cfg = dict(bench.PRESETS[args.config])
    strong = cfg.get("strong", False)
    rows = cfg["grid"] if strong else cfg["grid"] * args.gpus
    spinup = bench.spinup_for(cfg, args.gpus)
    nx = cfg["grid"]
    inp = bench.make_inp(nx, cfg["route_step"], cfg["variable_step"], cfg["pollutants"], cfg["diameter"], cfg["q"],
                         rows=rows)
    key = bench.workload_name(args.config, cfg, rows)
    s = swmm5.SWMM()
    d = "/tmp/swmm_bench"
    assert s.open(inp, os.path.join(d, "cal.rpt"), os.path.join(d, "cal.out")) == 0, s.getError()
    assert s.start(False) == 0, s.getError()
    backend = s.backend()

    def window():
        """Time --steps steps: per-iteration stats, kernel times, node work."""
        s.set_timing(True)
        assert s.run_steps(args.steps)[0] == 0, s.getError()
        out = (s.kernel_times(), s.iteration_stats(), s.node_work(), s.counters(), s.node_work(conduits=True))
        s.set_timing(False)
        return out

    def sparse(its):
        """Mean live node updates and us per launch pair over iterations k >= 3."""
        ks = [k for k in range(3, len(its)) if its[k][0] > 0]
        n = sum(its[k][0] for k in ks)
        if not n:
            return 0.0, 0.0, 0.0
        return (sum(its[k][3] for k in ks) / n, 1000.0 * sum(its[k][5] + its[k][6] for k in ks) / n, n)

    early = int(args.early_frac * spinup)
    assert s.run_steps(early)[0] == 0, s.getError()
    _, itsA, _, _, _ = window()
    assert s.run_steps(max(spinup - early - args.steps, 0) + args.warmup)[0] == 0, s.getError()
    kt, its, nw, c, cw = window()
    s.end()
    s.close()
    nN = nw.size
    row_updates = nw[:rows * nx].reshape(rows, nx).sum(axis=1) / args.steps
    row_conduit_updates = cw[:rows * nx].reshape(rows, nx).sum(axis=1) / args.steps
    uA, tA, _ = sparse(itsA)
    uB, tB, nB = sparse(its)
    reliable = uB - uA > 0.1 * max(uB, 1.0) and tB > tA
    b = (tB - tA) / (uB - uA) if reliable else 0.0
    f = tB - b * uB
    # per node and step: iterations 0 and 1 and the step end
    full_ms = sum(its[k][5] + its[k][6] for k in range(min(2, len(its)))) + kt["step_end"][1]
    c_node_us = 1000.0 * full_ms / args.steps / nN
    rec = {"config": args.config, "ranks_grid": args.gpus, "rows": rows, "nx": nx, "nodes": int(nN),
           "spinup": spinup, "warmup": args.warmup, "steps": args.steps,
           "iterations_per_step": round(c["iterations"] / max(c["steps"], 1), 3),
           "c_node_us_per_step": c_node_us,
           "sparse_us": {"window_A": {"start_step": early, "updates": round(uA, 1), "us": round(tA, 2)},
                         "window_B": {"start_step": spinup + args.warmup, "updates": round(uB, 1),
                                      "us": round(tB, 2)},
                         "floor_per_launch_pair": round(f, 2), "b_per_update": b, "reliable": bool(reliable)},
           "lambda": (b / c_node_us) if c_node_us > 0 else 0.0,
           "sparse_updates_per_step": float(row_updates.sum()),
           "row_updates": [round(float(x), 3) for x in row_updates],
           "row_conduit_updates": [round(float(x), 3) for x in row_conduit_updates],
           "backend": backend,
           "source": "tools/calibrate_partition.py --config %s --gpus %d --steps %d" % (args.config, args.gpus,
                                                                                       args.steps)}
    db = json.load(open(OUT)) if os.path.exists(OUT) else {}
    db[key] = rec
    with open(OUT, "w") as f:
        json.dump(db, f, indent=1)
    print(json.dumps({k: v for k, v in rec.items() if not k.startswith("row_")}))


if __name__ == "__main__":
    main()
