#!/usr/bin/env python3
"""Benchmark: dynamic-wave link-updates/s of the MI355X routing engine.

One "step" is one swmm_step (one full dynamic-wave routing step: the Picard
loop over all conduits and nodes plus per-step accounting) on the synthetic
Manhattan grid of SURVEY.md section 8(d), driven through the engine's C ABI.
Inputs are resident in HBM before the timed region (swmm_start uploads them).

    value = sum over timed steps of (true conduits x Picard iterations)
            / wall time of the K timed steps        (max over ranks, all ranks)

Default workload (N=1): 707 x 707 grid = 998,285 conduits / 499,850 nodes,
DYNWAVE, 1 s fixed routing step (BASELINE.json configs[1] scaled to the 1M
conduits the north_star target is quoted on; --grid 224 gives configs[1]).

Extra JSON objects:
  roofline      dominant kernel (link momentum) algorithmic bytes per launch
                (byte model in DESIGN.md, from swmmx_getKernelBytes) divided
                by its average HIP-event duration on the routing stream;
                peak 8000 GB/s (MI355X HBM3E spec).  "traffic" = PMC bytes
                from profiles/ when supplied with --traffic.
  cpu_baseline  the CPU restatement (oracle/, "port") timed on this host's
                cores on a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "stormwater-management-model_amd")
sys.path.insert(0, PKG)

METRIC = ("dynamic-wave link-updates/sec on synthetic grid net at 1/2/4/8 GPUs; HBM %peak")
HBM_PEAK_GBS = 8000.0


def make_inp(nx, route_step, variable_step, pollutants, diameter, q):
    import netgen
    d = os.path.join("/tmp", "swmm_bench")
    os.makedirs(d, exist_ok=True)
    name = "grid%d_rs%g_vs%g_p%d_d%g_q%g.inp" % (nx, route_step, variable_step, pollutants,
                                                  diameter, q)
    path = os.path.join(d, name)
    if not os.path.exists(path):
        tmp = path + ".%d.tmp" % os.getpid()
        netgen.write_grid(tmp, nx, nx, route_step=route_step, variable_step=variable_step,
                          pollutants=pollutants, diameter=diameter, q=q,
                          end_time="23:00:00", report_all=False)
        os.replace(tmp, path)
    return path


def cpu_baseline(inp, steps, q, route_step):
    """Time the oracle (plain-C restatement, single thread) on the same grid."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import swmm5
    from _dumpio import read_dump
    from _oracle import oracle_from_dump
    s = swmm5.SWMM()
    tmpd = "/tmp/swmm_bench"
    os.makedirs(tmpd, exist_ok=True)
    assert s.open(inp, os.path.join(tmpd, "cpu.rpt"), os.path.join(tmpd, "cpu.out")) == 0
    assert s.start_host() == 0
    dump = os.path.join(tmpd, "cpu_init_%d.bin" % os.getpid())
    s.export_state(dump)
    nL = s.getCount(swmm5.LINK)
    s.close()
    o = oracle_from_dump(read_dump(dump))
    os.remove(dump)
    lat = np.full(o.nN, q)
    lat[-1] = 0.0                       # the outfall has no DWF
    o.d("node.latIn")[:] = lat
    t0 = time.perf_counter()
    iters = 0
    for _ in range(steps):
        iters += o.step(route_step)
    dt = time.perf_counter() - t0
    return nL * iters / dt, iters / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--grid", type=int, default=707)
    ap.add_argument("--route-step", type=float, default=1.0)
    ap.add_argument("--variable-step", type=float, default=0.0)
    ap.add_argument("--pollutants", type=int, default=0)
    ap.add_argument("--diameter", type=float, default=1.5)
    ap.add_argument("--q", type=float, default=0.02)
    ap.add_argument("--cpu-steps", type=int, default=40)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--timing-steps", type=int, default=10)
    ap.add_argument("--traffic", type=float, default=None,
                    help="HBM bytes per link-momentum launch from rocprofv3 PMC (profiles/)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    import swmm5
    inp = make_inp(args.grid, args.route_step, args.variable_step, args.pollutants,
                   args.diameter, args.q)
    s = swmm5.SWMM()
    s.set_device(local)
    tmpd = "/tmp/swmm_bench"
    err = s.open(inp, os.path.join(tmpd, "r%d.rpt" % rank), os.path.join(tmpd, "r%d.out" % rank))
    if err:
        raise SystemExit("swmm_open failed: %s" % (s.getError(),))
    err = s.start(False)
    if err:
        raise SystemExit("swmm_start failed: %s" % (s.getError(),))
    backend = s.backend()
    if not backend.startswith("hip:"):
        raise SystemExit("HIP backend not active: " + backend)
    nL = s.getCount(swmm5.LINK)
    nN = s.getCount(swmm5.NODE)

    err, _ = s.run_steps(args.warmup)
    assert err == 0, s.getError()
    c0 = s.counters()                       # synchronises the device
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    err, _ = s.run_steps(args.steps)
    c1 = s.counters()                       # synchronises the device
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    assert err == 0, s.getError()
    elapsed = t1 - t0
    iters = c1["iterations"] - c0["iterations"]
    updates = float(nL) * float(iters)
    if dist:
        import torch
        t = torch.tensor([elapsed, updates], dtype=torch.float64)
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum[1:], op=dist.ReduceOp.SUM)
        elapsed, updates = float(tmax[0]), float(tsum[1])

    # per-kernel timing (HIP events on the routing stream), eager launches
    s.set_timing(True)
    err, _ = s.run_steps(args.timing_steps)
    kt = s.kernel_times()
    kb = s.kernel_bytes()
    s.set_timing(False)
    s.end()
    s.close()

    link_n, link_ms = kt["link_momentum"]
    node_n, node_ms = kt["node_update"]
    link_avg_s = (link_ms / 1000.0) / max(link_n, 1)
    node_avg_s = (node_ms / 1000.0) / max(node_n, 1)
    achieved = kb["link_momentum"] / link_avg_s / 1e9 if link_avg_s > 0 else 0.0
    roof = {
        "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": args.traffic,
        "kernel": "k_link (link momentum, dwflow_findConduitFlow)",
        "avg_launch_us": round(link_avg_s * 1e6, 2),
        "bytes_per_launch": kb["link_momentum"],
        "node_update": {"avg_launch_us": round(node_avg_s * 1e6, 2),
                        "achieved_GBs": round(kb["node_update"] / node_avg_s / 1e9, 2) if node_avg_s > 0 else 0.0},
    }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        rate, ipc = cpu_baseline(inp, args.cpu_steps, args.q, args.route_step)
        cpu = {"value": round(rate, 1), "unit": "link-updates/s", "cores": 1, "kind": "port",
               "sample": "%d routing steps of the same %dx%d grid from its initial state, "
                         "oracle/dw_oracle.c single-threaded (%.2f iterations/step)"
                         % (args.cpu_steps, args.grid, args.grid, ipc)}

    if rank == 0:
        value = updates / elapsed
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "link-updates/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic",
            "config": {"workload": "manhattan_grid_%dx%d_DYNWAVE_%s" % (
                           args.grid, args.grid,
                           "fixed%gs" % args.route_step if args.variable_step == 0 else
                           "variable%g" % args.variable_step),
                       "conduits": nL, "nodes": nN, "pollutants": args.pollutants,
                       "iterations_per_step": round(iters / args.steps, 3),
                       "parallelism": "replicas" if world > 1 else "single",
                       "backend": backend},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
