#!/usr/bin/env python3
"""Partition weights for bench.py's multi-GPU runs, measured on one GPU.

The sparse Picard iterations (k >= 2) follow the surcharge, which builds up
next to the outlet: contiguous row strips of equal size leave the strip
holding the outlet with several times the others' sparse work (DESIGN.md
section 6).  This tool runs a bench workload's whole grid on one GPU through
its spin-up, then times --steps steps (timing mode) and records

  * per grid row, the node updates per step in iterations k >= 2
    (swmmx_getNodeWork: the measured sparse work, node by node);
  * the cost of a full-pass node per step (iterations 0 and 1 and the step
    end, per node) and the marginal cost of one sparse node update (a least-
    squares fit t_k = a + b u_k over the iterations k >= 2 of the window:
    the launch floor a is paid by every rank alike and is not balanced).

bench.py --balance (the default with several ranks) then weighs node i of
row r as 1 + (b / c_full) * u_r / nx, and swmmx_setPartitionWeights cuts the
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

import bench  # noqa: E402
import swmm5  # noqa: E402

OUT = os.path.join(ROOT, "profiles", "partition_weights.json")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4m", choices=sorted(bench.PRESETS))
    ap.add_argument("--gpus", type=int, default=2, help="rank count whose grid (weak scaling) and spin-up apply")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
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
    assert s.run_steps(spinup + args.warmup)[0] == 0, s.getError()
    s.set_timing(True)
    assert s.run_steps(args.steps)[0] == 0, s.getError()
    kt = s.kernel_times()
    its = s.iteration_stats()
    nw = s.node_work()
    c = s.counters()
    s.set_timing(False)
    s.end()
    s.close()
    nN = nw.size
    row_updates = nw[:rows * nx].reshape(rows, nx).sum(axis=1) / args.steps
    # full passes per node per step: iterations 0 and 1 and the step end (ms)
    full_ms = sum(its[k][5] + its[k][6] for k in range(min(2, len(its)))) + kt["step_end"][1]
    c_full_us = 1000.0 * full_ms / args.steps / nN
    # sparse iterations: t_k = a + b u_k over k >= 2 (per launch pair, us)
    ks = [k for k in range(2, len(its)) if its[k][0] > 0]
    u = np.array([its[k][3] / its[k][0] for k in ks])
    t = np.array([1000.0 * (its[k][5] + its[k][6]) / its[k][0] for k in ks])
    if len(ks) >= 2 and np.ptp(u) > 0:
        b, a = np.polyfit(u, t, 1)
    else:
        a, b = 0.0, (t.sum() / max(u.sum(), 1.0)) if len(ks) else 0.0
    b = max(float(b), 0.0)
    rec = {"config": args.config, "ranks_grid": args.gpus, "rows": rows, "nx": nx, "nodes": int(nN),
           "spinup": spinup, "warmup": args.warmup, "steps": args.steps,
           "iterations_per_step": round(c["iterations"] / max(c["steps"], 1), 3),
           "c_full_us_per_node": c_full_us, "sparse_fit_us": {"a": float(a), "b_per_update": b},
           "lambda": (b / c_full_us) if c_full_us > 0 else 0.0,
           "sparse_updates_per_step": float(row_updates.sum()),
           "row_updates": [round(float(x), 3) for x in row_updates],
           "backend": backend,
           "source": "tools/calibrate_partition.py --config %s --gpus %d --steps %d" % (args.config, args.gpus,
                                                                                       args.steps)}
    db = json.load(open(OUT)) if os.path.exists(OUT) else {}
    db[key] = rec
    with open(OUT, "w") as f:
        json.dump(db, f, indent=1)
    print(json.dumps({k: v for k, v in rec.items() if k != "row_updates"}))


if __name__ == "__main__":
    main()
