#!/usr/bin/env python3
"""Benchmark: dynamic-wave link-updates/s of the MI355X routing engine.

One "step" is one swmm_step (one full dynamic-wave routing step: the Picard
loop over all conduits and nodes plus per-step accounting) on the synthetic
Manhattan grid of SURVEY.md section 8(d), driven through the engine's C ABI.
Inputs are resident in HBM before the timed region (swmm_start uploads them).

    value = sum over timed steps of (true conduits x Picard iterations)
            / wall time of the K timed steps        (max over ranks, all ranks)

Workloads (--config; BASELINE.json configs):
  1m_surcharge (default, configs[2]) 707 x 707 grid = 998,285 conduits /
        499,850 nodes, DYNWAVE, VARIABLE_STEP 0.75, ROUTING_STEP 5 s, 1.0-ft
        pipes, DWF 0.12 cfs per junction.  The run is first spun up for
        --spinup steps (untimed, outside warmup) so that 2-20 % of the
        junctions are surcharged in the timed window (fraction
        reported in config.surcharged_pct).
  1m_light  the same with 0.1 cfs (0.3-0.8 % surcharged; rounds 1-3's preset).
  1m_quality (configs[3]) the same plus 3 pollutants (advection + decay).
  100k (configs[1]) 224 x 224 grid = 99,905 conduits, fixed 1 s step.
  1m_fixed  707 x 707, fixed 1 s step, 1.5-ft pipes (no surcharge).
  4m (configs[4]) 1414 x 1414 grid = 3,995,965 conduits, the 1m_surcharge
        hydraulics; the same grid at every rank count (strong scaling), one
        row strip per rank.  The other presets scale weakly: N ranks route a
        (707 N) x 707 grid, one 707-row strip each.

Extra JSON objects:
  roofline      dominant kernel (link momentum) algorithmic bytes per launch
                (byte model in DESIGN.md, from swmmx_getKernelBytes) divided
                by its average HIP-event duration on the routing stream;
                peak 8000 GB/s (MI355X HBM3E spec).  "traffic" = PMC bytes
                per launch from profiles/ when supplied with --traffic.
  cpu_baseline  the CPU restatement (oracle/, "port") timed on this host's
                cores on a bounded sample of the same workload, continuing
                from the spun-up state.
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


PRESETS = {
    # 2-20 % of the junctions surcharged in the timed window.  At
    # q = 0.12 cfs the surcharged fraction grows from 2.2 % at step 700 to 9.0 %
    # at step 1000, then the grid floods (96 % by step 1100; profiles/
    # r04_regime_traj.txt); every step of the band runs all 8 Picard iterations
    # weak scaling (--gpus N routes a (707 N) x 707 grid, one 707-row strip per
    # rank): the surcharge front reaches the outlet later on the longer grids,
    # so the spin-up grows with N to keep the timed window at 4-5 %
    # surcharged (profiles/r05_regime_traj_weak.txt: 4.2 % at step 900 for
    # N = 2, 4.2 % at 950 for N = 4 and 4.1 % at 950 for N = 8)
    "1m_surcharge": dict(grid=707, route_step=5.0, variable_step=0.75, diameter=1.0, q=0.12,
                         pollutants=0, spinup=750, spinup_by_n={2: 900, 4: 950, 8: 950}),
    "1m_quality": dict(grid=707, route_step=5.0, variable_step=0.75, diameter=1.0, q=0.12,
                       pollutants=3, spinup=750, spinup_by_n={2: 900, 4: 950, 8: 950}),
    # the light-surcharge regime of rounds 1-3 (0.3-0.8 % surcharged; a few
    # thousand nodes stay live after iteration 1, 7.4 iterations per step)
    "1m_light": dict(grid=707, route_step=5.0, variable_step=0.75, diameter=1.0, q=0.1,
                     pollutants=0, spinup=400),
    "100k": dict(grid=224, route_step=1.0, variable_step=0.0, diameter=1.5, q=0.02,
                 pollutants=0, spinup=0),
    "1m_fixed": dict(grid=707, route_step=1.0, variable_step=0.0, diameter=1.5, q=0.02,
                     pollutants=0, spinup=0),
    # configs[4]: one 1414 x 1414 grid (3,995,965 conduits) whatever the rank
    # count, link-partitioned into row strips (strong scaling)
    # q = 0.12 cfs: 2.9 % surcharged at step 900, 4.7 % at 1000, flooded
    # (97 %) by step 1100 (profiles/r04_regime_traj_4m.txt)
    "4m": dict(grid=1414, route_step=5.0, variable_step=0.75, diameter=1.0, q=0.12,
               pollutants=0, spinup=850, strong=True),
}


def make_inp(nx, route_step, variable_step, pollutants, diameter, q, rows=None):
    """Grid .inp with `rows` x nx junctions (rows defaults to nx); row-major
    node order, so contiguous node blocks are row strips."""
    import netgen
    rows = rows or nx
    d = os.path.join("/tmp", "swmm_bench")
    os.makedirs(d, exist_ok=True)
    name = "grid%dx%d_rs%g_vs%g_p%d_d%g_q%g.inp" % (rows, nx, route_step, variable_step,
                                                     pollutants, diameter, q)
    path = os.path.join(d, name)
    if not os.path.exists(path):
        tmp = path + ".%d.tmp" % os.getpid()
        netgen.write_grid(tmp, rows, nx, route_step=route_step, variable_step=variable_step,
                          pollutants=pollutants, diameter=diameter, q=q,
                          end_time="23:00:00", report_all=False)
        os.replace(tmp, path)
    return path


def spinup_for(cfg, world):
    """the preset's spin-up for this rank count (weak scaling: the longer grid's
    own spin-up, nearest tabulated rank count below)"""
    spin = cfg["spinup"]
    if world > 1 and cfg.get("spinup_by_n"):
        keys = sorted(k for k in cfg["spinup_by_n"] if k <= world)
        if keys:
            spin = cfg["spinup_by_n"][keys[-1]]
    return spin


def workload_name(config, cfg, rows):
    return "%s: manhattan_grid_%dx%d_DYNWAVE_%s_D%gft_q%gcfs_P%d" % (
        config, rows, cfg["grid"],
        "fixed%gs" % cfg["route_step"] if cfg["variable_step"] == 0 else
        "variable%g_max%gs" % (cfg["variable_step"], cfg["route_step"]),
        cfg["diameter"], cfg["q"], cfg["pollutants"])


def partition_weights(workload, rows, nx, n_nodes, lam=None):
    """Per-node weights from profiles/partition_weights.json (tools/
    calibrate_partition.py: the workload's per-row sparse node updates per
    step measured on one GPU -- node updates plus the updates of the
    conduits whose node1 lies in the row -- and the marginal cost of a sparse
    update relative to a full-pass node): node i of row r weighs
    1 + lambda u_r / nx (lam overrides the record's lambda), the outfall 1.  None when no record
    matches this grid."""
    path = os.path.join(ROOT, "profiles", "partition_weights.json")
    if not os.path.exists(path):
        return None, None
    rec = json.load(open(path)).get(workload)
    if not rec or rec.get("rows") != rows or rec.get("nx") != nx or rec.get("nodes") != n_nodes:
        return None, None
    import numpy as np
    w = np.ones(n_nodes)
    ru = np.asarray(rec["row_updates"], dtype=np.float64)
    if "row_conduit_updates" in rec:          # + the conduits' updates, charged to their node1 (their owner)
        ru = ru + np.asarray(rec["row_conduit_updates"], dtype=np.float64)
    if lam is None:                           # an unreliable calibration (no lambda): weigh updates 1:1
        lam = rec["lambda"] if rec.get("lambda", 0.0) > 0.0 else 1.0
    w[:rows * nx] = 1.0 + lam * np.repeat(ru / nx, nx)
    return w, rec


def _record(name, workload, backend):
    """profiles/<name> entry for this workload, only when it was measured on
    the same build inputs (swmm5.kernel_source_sha: every engine source,
    header and the Makefile's flags) and the same device"""
    import swmm5
    tp = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(tp):
        return None
    rec = json.load(open(tp)).get(workload)
    if not rec or rec.get("src_sha") != swmm5.kernel_source_sha() or rec.get("backend") != backend:
        return None
    return rec


def pmc_record(workload, backend):
    """profiles/pmc_traffic.json entry for this workload (tools/pmc_summary.py)"""
    return _record("pmc_traffic.json", workload, backend)


def same_regime(rec_window, window):
    """A profile record taken over another timed window of the same regime:
    the same spin-up (the window's surcharge level), any steps / warm-up (the
    driver runs --steps 20 --warmup 5, the profiles may be longer)"""
    return rec_window is None or (len(rec_window) == 3 and rec_window[0] == window[0])


def timing_record(workload, window, backend):
    """profiles/kernel_timing.json entry (tools/rocprof_summary.py): the
    in-graph k_link<first> duration over a timed window of this workload in
    the same regime (same_regime)"""
    rec = _record("kernel_timing.json", workload, backend)
    if not rec or not same_regime(rec.get("window"), window):
        return None
    return rec


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_threads():
    """The host cores this process may use: every CPU of the affinity mask
    (BASELINE.md's THREADS = nproc), bounded only by OMP_NUM_THREADS when the
    machine sets it -- the GPU pool gives each one-GPU box a 16-CPU share of
    its host that way (os.cpu_count() there shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, n)


def cpu_baseline(dump, steps, q, route_step, variable, threads=1):
    """Time the oracle (plain-C restatement) from a state dump; threads > 1
    runs its per-link and per-node loops on OpenMP threads (same bits)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _dumpio import read_dump
    from _oracle import oracle_resume
    o = oracle_resume(read_dump(dump))
    o.opt("threads", threads)
    lat = np.full(o.nN, q)
    lat[-1] = 0.0                       # the outfall has no DWF
    o.d("node.latIn")[:] = lat
    t0 = time.perf_counter()
    iters = 0
    for _ in range(steps):
        dt = o.routing_step(route_step) if variable else route_step
        iters += o.step(dt)
    dt = time.perf_counter() - t0
    return o.nL * iters / dt, iters / steps, dt


def ref_baseline(threads, seconds=10.0):
    """The reference solver itself (oracle/_ref/ref_timing: EPA SWMM 5.2.4
    compiled from its own sources, checker infrastructure) on configs[1]'s
    100k grid (224 x 224, fixed 1 s step), on 1 thread and on `threads`
    (its THREADS option): `seconds` of its step loop each, timed inside the
    harness from swmm_start to the last step (parse excluded).  None when the
    harness was not built (no /root/reference where the oracle was built)."""
    import subprocess
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_timing")
    if not os.path.exists(exe):
        return None
    import netgen
    d = os.path.join("/tmp", "swmm_bench")
    os.makedirs(d, exist_ok=True)
    legs = {}
    for nt in sorted({1, threads}):
        inp = os.path.join(d, "ref100k_t%d.inp" % nt)
        netgen.write_grid(inp, 224, 224, route_step=1.0, variable_step=0.0, diameter=1.5, q=0.02,
                          end_time="23:00:00", report_all=False, threads=nt)
        out = subprocess.run([exe, inp, os.path.join(d, "ref%d.rpt" % nt), os.path.join(d, "ref%d.out" % nt),
                              str(seconds), "1000000"], capture_output=True, text=True, timeout=300)
        r = json.loads(out.stdout.strip().splitlines()[-1])
        if r["error"] or r["iterations_per_step"] <= 0:
            return None
        r["value"] = r["links"] * r["iterations_per_step"] * r["steps"] / r["step_s"]
        legs[nt] = r
    one, many = legs[1], legs[threads]
    return {"value": round(many["value"], 1), "unit": "link-updates/s", "cores": threads, "kind": "reference",
            "single_thread": {"value": round(one["value"], 1), "cores": 1, "steps": one["steps"],
                              "seconds": round(one["step_s"], 2)},
            "parse_s": round(many["open_s"], 2),
            "iterations_per_step": many["iterations_per_step"],
            "sample": "EPA SWMM 5.2.4 itself (oracle/_ref/libswmm5_ref.so from /root/reference's sources, -O3 "
                      "OpenMP) on configs[1]'s 224 x 224 grid (99,905 conduits, fixed 1 s step): %d and %d "
                      "steps from swmm_start in %.1f s on %d threads and %.1f s on 1 thread (THREADS option; "
                      "swmm_open's parse, %.2f s, excluded); Picard iterations from its report"
                      % (many["steps"], one["steps"], many["step_s"], threads, one["step_s"], many["open_s"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", choices=sorted(PRESETS), default="1m_surcharge")
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--spinup", type=int, default=None)
    ap.add_argument("--q", type=float, default=None, help="override the preset's DWF per junction (cfs)")
    ap.add_argument("--diameter", type=float, default=None, help="override the preset's pipe diameter (ft)")
    ap.add_argument("--cpu-steps", type=int, default=60, help="routing steps of the CPU port's leg (~6 s on 16 "
                                                                   "cores, ~15 s on one)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--timing-steps", type=int, default=10)
    ap.add_argument("--kernel-reps", type=int, default=20)
    ap.add_argument("--exchange", choices=["ipc", "rccl", "host"], default="ipc",
                    help="multi-GPU transport: ipc = each rank's kernels store the ghost-link values, "
                         "convergence flags and Courant limits into its peers' memory (no collective inside a "
                         "step; falls back to rccl if its start-up handshake fails); rccl = captured ncclSend/"
                         "ncclRecv + ncclAllReduce; host = gloo through the host (rehearsal on one GPU)")
    ap.add_argument("--rccl-1rank", action="store_true",
                    help="one GPU through the partitioned RCCL code path (captured neighbour send/recv and "
                         "flag all-reduce every Picard iteration): the in-graph cost of the collectives")
    ap.add_argument("--no-stream", dest="stream", action="store_false",
                    help="skip the STREAM-triad measurement of the achievable HBM bandwidth")
    ap.add_argument("--balance", choices=["auto", "weighted", "off"], default="auto",
                    help="several ranks, when the workload has a record of its measured sparse work "
                         "(profiles/partition_weights.json, tools/calibrate_partition.py): auto = two regions "
                         "(the surcharged band and the rest, each shared equally), weighted = contiguous blocks "
                         "of equal weight; off = row strips of equal node count")
    ap.add_argument("--traffic", type=float, default=None,
                    help="HBM bytes per link-momentum launch from rocprofv3 PMC (profiles/)")
    args = ap.parse_args()
    cfg = dict(PRESETS[args.config])
    if args.grid is not None:
        cfg["grid"] = args.grid
    if args.spinup is not None:
        cfg["spinup"] = args.spinup
    if args.q is not None:
        cfg["q"] = args.q
    if args.diameter is not None:
        cfg["diameter"] = args.diameter

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.spinup is None:
        # the weak-scaling grid's own spin-up (nearest tabulated rank count below)
        cfg["spinup"] = spinup_for(cfg, world)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")   # single-node RCCL bootstrap

    import swmm5
    # weak scaling: world row strips of grid x grid junctions (about 1M conduits
    # per GPU), link-partitioned, one RCCL all-reduce per Picard iteration;
    # strong scaling (4m): one grid x grid network split into world strips
    strong = cfg.get("strong", False)
    rows = cfg["grid"] if strong else cfg["grid"] * world
    if rank == 0:
        inp = make_inp(cfg["grid"], cfg["route_step"], cfg["variable_step"], cfg["pollutants"],
                       cfg["diameter"], cfg["q"], rows=rows)
    if dist:
        dist.barrier()
        inp = make_inp(cfg["grid"], cfg["route_step"], cfg["variable_step"], cfg["pollutants"],
                       cfg["diameter"], cfg["q"], rows=rows)
    s = swmm5.SWMM()
    s.set_device(local)
    if world > 1:
        import torch
        idt = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            idt = torch.frombuffer(bytearray(s.nccl_unique_id().ljust(128, b"\0")), dtype=torch.uint8)
        dist.broadcast(idt, 0)
        s.set_partition(rank, world, bytes(idt.numpy().tobytes()))
    elif args.rccl_1rank:
        s.set_partition(0, 1, s.nccl_unique_id())
    balance = None
    if world > 1 and args.balance != "off":
        # node i weighs 1 + lambda u_i (u: its measured sparse updates per
        # step, node and conduits; lambda: a sparse update's cost relative to
        # a full-pass node, both from the calibration record).  auto: two
        # regions -- the surcharged band, dealt in 2R blocks 0..R-1, R-1..0,
        # and the rest in R blocks, all of equal weight; weighted: one
        # contiguous block of equal weight per rank
        n_nodes = rows * cfg["grid"] + 1
        w, balance = partition_weights(workload_name(args.config, cfg, rows), rows, cfg["grid"], n_nodes)
        if w is not None:
            s.set_partition_weights(w)
            if args.balance == "auto":
                s.set_partition_mode("two_region")
    if world > 1 and args.exchange in ("host", "ipc"):
        # host transport (gloo through torch.distributed): the rehearsal of
        # the multi-rank path with several ranks on one GPU; the IPC transport
        # is bootstrapped over the same callback (IPC handles at swmm_start,
        # the result gathers at report times and at swmm_end)
        def xchg(arr, op):
            t = torch.from_numpy(arr)
            dist.all_reduce(t, op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MIN)
        s.set_exchange(xchg)
        if args.exchange == "ipc":
            s.set_transport("ipc")
    tmpd = "/tmp/swmm_bench"
    err = s.open(inp, os.path.join(tmpd, "r%d.rpt" % rank), os.path.join(tmpd, "r%d.out" % rank))
    if err:
        raise SystemExit("swmm_open failed: %s" % (s.getError(),))
    err = s.start(False)
    if err:
        raise SystemExit("swmm_start failed: %s" % (s.getError(),))
    backend = s.backend()
    transport = s.transport()
    if not backend.startswith("hip:"):
        raise SystemExit("HIP backend not active: " + backend)
    nL = s.getCount(swmm5.LINK)
    nN = s.getCount(swmm5.NODE)
    nL_rank = int((s.owners(swmm5.LINK) == rank).sum()) if world > 1 else nL
    # this rank's layout: owned nodes, held nodes (owned + replicas), ghost links
    layout = ([int((s.owners(swmm5.NODE) == rank).sum()), int(s.partition_array("lnode").size),
               int(s.partition_array("lghost").size)] if world > 1 else [nN, nN, 0])

    if cfg["spinup"]:
        err, _ = s.run_steps(cfg["spinup"])
        assert err == 0, s.getError()
    err, _ = s.run_steps(args.warmup)
    assert err == 0, s.getError()
    c0 = s.counters()                       # synchronises the device
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    err, t_days = s.run_steps(args.steps)
    c1 = s.counters()                       # synchronises the device
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    assert err == 0, s.getError()
    elapsed = t1 - t0
    iters = c1["iterations"] - c0["iterations"]
    nonconv = c1["nonconverged"] - c0["nonconverged"]
    updates = float(nL_rank) * float(iters)          # this rank's conduits
    if dist:
        import torch
        t = torch.tensor([elapsed, updates], dtype=torch.float64)
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum[1:], op=dist.ReduceOp.SUM)
        elapsed, updates = float(tmax[0]), float(tsum[1])
    depth = s.get_array("node.newDepth")
    if world > 1:
        # every rank's owned junctions (the whole grid, not rank 0's strip)
        import torch
        mine = s.owners(swmm5.NODE)[:-1] == rank
        cnt = torch.tensor([float((depth[:-1][mine] > cfg["diameter"]).sum()), float(mine.sum())],
                           dtype=torch.float64)
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
        surcharged = float(cnt[0] / cnt[1]) * 100.0
    else:
        surcharged = float((depth[:-1] > cfg["diameter"]).mean()) * 100.0

    dump = None
    if rank == 0 and world == 1 and not args.no_cpu:
        dump = os.path.join(tmpd, "cpu_state_%d.bin" % os.getpid())
        s.export_state(dump)

    # per-kernel timing (HIP events on the routing stream), eager launches
    s.set_timing(True)
    err, _ = s.run_steps(args.timing_steps)
    kt = s.kernel_times()
    kb = s.kernel_bytes()
    its = s.iteration_stats()
    tw = s.counters()
    s.set_timing(False)
    # dominant kernel alone: back-to-back launches between two HIP events on
    # the routing stream (per-launch dispatch gaps amortised); after the timed
    # run because it advances the state
    b2b_us = s.time_kernel(0, args.kernel_reps) if args.kernel_reps > 0 else 0.0
    s.end()
    s.close()
    # the achievable HBM bandwidth of this GPU: STREAM triad over
    # three 512 MB fp64 arrays, HIP events, outside any profiler
    stream = s.stream_triad(64 << 20, 20) if args.stream else None

    workload = workload_name(args.config, cfg, rows)

    def avg_us(name):
        n, ms = kt[name]
        return 1000.0 * ms / n if n else 0.0

    def gbs(name):
        us = avg_us(name)
        return kb[name] / (us * 1e-6) / 1e9 if us > 0 else 0.0

    first_bytes = kb["link_momentum_first"]
    eager_us = avg_us("link_momentum_first")          # in-step, kernel execution timestamps
    first_us, timing = eager_us, ("in-step: %d routing steps launched eagerly, each kernel with "
                                  "hipExtLaunchKernelGGL start/stop events (the kernel's own execution "
                                  "timestamps, as rocprofv3's kernel trace)" % kt["link_momentum_first"][0])
    trec = timing_record(workload, [cfg["spinup"], args.warmup, args.steps], backend)
    if trec:                               # the graph launches' own duration (rocprofv3, same window)
        first_us = trec["avg_launch_us"]
        timing = ("in-graph: rocprofv3 --kernel-trace average of the %d graph launches of %s in a timed "
                  "window of this workload (spin-up, warm-up, steps = %s; %s)"
                  % (trec["launches"], trec["kernel"], trec.get("window"), trec["source"]))
    achieved = first_bytes / (first_us * 1e-6) / 1e9
    it_n = tw["timed_iters1"]               # timed iterations >= 1 (either step graph)
    n0 = kt["link_momentum_first"][0]
    bypass = None
    eff = None                             # conduit updates not bypassed / nominal updates
    if it_n:
        bypass = 100.0 * (1.0 - tw["timed_updated"] / (it_n * tw["streaming_conduits"]))
        eff = (n0 * tw["streaming_conduits"] + tw["timed_updated"]) / ((n0 + it_n) * tw["streaming_conduits"])
    regather = None
    if tw.get("timed_gather_iters"):
        regather = 100.0 * tw["timed_gathered"] / (tw["timed_gather_iters"] * tw["nodes"])
    traffic = args.traffic
    traffic_src = "--traffic" if traffic is not None else None
    step_bytes = None
    rec = None
    if traffic is None:                    # PMC measurement committed for this workload
        rec = pmc_record(workload, backend)
        if rec:
            traffic, traffic_src = rec["bytes_per_launch"], rec["source"]
            step_bytes = rec.get("step_bytes")
            # the PMC pass must have measured this same window (same steps, same
            # regime); otherwise its per-step bytes describe another workload
            if not same_regime(rec.get("window"), [cfg["spinup"], args.warmup, args.steps]) or \
                    abs(rec.get("iterations_per_step", 0) - iters / args.steps) > 1e-6:
                step_bytes = None
    step_s = elapsed / args.steps
    roof = {
        "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        # the achievable peak on this box (STREAM triad, best of 20 launches)
        # and the kernel's fraction of it
        "peak_measured": None if not stream else round(stream["triad_best_GBs"], 1),
        "frac_measured": None if not stream else round(achieved / stream["triad_best_GBs"], 4),
        "stream": None if not stream else {
            "triad_best_GBs": round(stream["triad_best_GBs"], 1), "triad_avg_GBs": round(stream["triad_avg_GBs"], 1),
            "copy_best_GBs": round(stream["copy_best_GBs"], 1),
            "kernel": "a[i] = b[i] + s c[i], fp64, 16-byte lanes, 3 x 512 MB arrays, 8 workgroups per CU "
                      "(stormwater-management-model_amd/csrc/stream.hip)"},
        "traffic": traffic,
        "traffic_source": traffic_src,
        # whole step: PMC HBM bytes per routing step of the same timed window
        # (same workload, steps, iterations and kernel source) over the
        # measured step time
        "step_traffic": step_bytes,
        "step_traffic_iterations_per_step": None if not step_bytes else rec.get("iterations_per_step"),
        "step_achieved": None if not step_bytes else round(step_bytes / step_s / 1e9, 2),
        "step_frac": None if not step_bytes else round(step_bytes / step_s / 1e9 / HBM_PEAK_GBS, 4),
        "step_frac_measured": None if not (step_bytes and stream)
        else round(step_bytes / step_s / 1e9 / stream["triad_best_GBs"], 4),
        "kernel": "k_link<first> (Picard iteration 0 link momentum, dwflow_findConduitFlow, "
                  "every conduit)",
        "avg_launch_us": round(first_us, 2),
        "timing": timing,
        "bytes_per_launch": first_bytes,
        "other_kernels": {
            "k_link<first> in-step eager": {
                "avg_launch_us": round(eager_us, 2),
                "achieved_GBs": round(first_bytes / (eager_us * 1e-6) / 1e9, 1) if eager_us else None,
                "note": "this run: %d routing steps launched eagerly, each kernel between "
                        "hipExtLaunchKernelGGL start/stop events" % kt["link_momentum_first"][0]},
            "k_link<first> back-to-back": {
                "avg_launch_us": round(b2b_us, 2),
                "achieved_GBs": round(first_bytes / (b2b_us * 1e-6) / 1e9, 1) if b2b_us else None,
                "note": "%d back-to-back launches of a separately named instantiation on the live "
                        "state (caches warm from the previous launch); secondary" % args.kernel_reps},
            "k_node<first>": {"avg_launch_us": round(avg_us("node_update_first"), 2),
                              "achieved_GBs": round(gbs("node_update_first"), 1)},
            "k_link iterations>=1": {"avg_launch_us": round(avg_us("link_momentum_iter"), 2),
                                     "achieved_GBs": round(gbs("link_momentum_iter"), 1),
                                     "bypassed_pct": None if bypass is None else round(bypass, 2)},
            "k_node iteration 1": {"avg_launch_us": round(avg_us("node_update_iter1"), 2),
                                   "achieved_GBs": round(gbs("node_update_iter1"), 1)},
            "k_node iterations>=2": {"avg_launch_us": round(avg_us("node_update_iter2plus"), 2),
                                     "achieved_GBs": round(gbs("node_update_iter2plus"), 1),
                                     "regathered_pct": None if regather is None else round(regather, 2)},
            "k_step_end+k_finalize": {"avg_launch_us": round(avg_us("step_end"), 2),
                                      "achieved_GBs": round(gbs("step_end"), 1)},
        },
    }
    if kt.get("sparse_tail", (0, 0))[0]:
        roof["other_kernels"]["k_sparse+k_unfreeze"] = {
            "avg_launch_us": round(avg_us("sparse_tail"), 2),
            "launches": int(kt["sparse_tail"][0]),
            "note": "Picard iterations >= 2 of a sparse-graph step in one workgroup, then the frozen "
                    "junctions' final depths (per-iteration work in per_iteration)"}
    # per Picard iteration of the timing-mode steps: how much work each one
    # does and what its two launches cost
    per_iter = []
    for k, r in enumerate(its):
        if r[0] > 0:
            per_iter.append({"k": k, "runs": int(r[0]), "conduits_updated": round(r[1] / r[0]),
                             "nodes_updated": round(r[3] / r[0]), "nodes_relax_only": round(r[4] / r[0]),
                             "nodes_gathered": round(r[2] / r[0]),
                             "k_link_us": round(1000.0 * r[5] / r[0], 2),
                             "k_node_us": round(1000.0 * r[6] / r[0], 2)})
    roof["per_iteration"] = per_iter
    if dist:
        # each rank's sparse work (iterations k >= 2): the load balance of the
        # strips (the surcharged region sits next to the outlet, on the last one)
        mine_w = [round(sum(x["conduits_updated"] for x in per_iter if x["k"] >= 2)),
                  round(sum(x["nodes_updated"] for x in per_iter if x["k"] >= 2)),
                  *layout]
        allw = [None] * world
        dist.all_gather_object(allw, mine_w)
        roof["per_rank_sparse_work"] = {"conduits_updated_k>=2": [w[0] for w in allw],
                                        "nodes_updated_k>=2": [w[1] for w in allw],
                                        "owned_nodes": [w[2] for w in allw], "held_nodes": [w[3] for w in allw],
                                        "ghost_links": [w[4] for w in allw]}
    if world > 1 and kt.get("ghost_exchange", (0, 0))[0]:
        # the per-iteration exchanges on the routing stream (timing-mode
        # steps): their cost per Picard iteration on this rank
        roof["other_kernels"]["ghost_exchange"] = {
            "avg_us": round(avg_us("ghost_exchange"), 2), "launches": int(kt["ghost_exchange"][0]),
            "note": "per Picard iteration: pack .. unpack of the strip neighbours' ghost-link values (%s)" % transport}
        roof["other_kernels"]["flag_exchange"] = {
            "avg_us": round(avg_us("flag_exchange"), 2), "launches": int(kt["flag_exchange"][0]),
            "note": "per Picard iteration: the convergence flag reduced over every rank (%s)" % transport}
    if cfg["pollutants"]:
        roof["other_kernels"]["k_qual_node+k_qual_link"] = {
            "avg_launch_us": round(avg_us("quality"), 2), "achieved_GBs": round(gbs("quality"), 1)}

    cpu = None
    if dump:
        nt = cpu_threads()
        rate1, ipc, secs1 = cpu_baseline(dump, args.cpu_steps, cfg["q"], cfg["route_step"],
                                         cfg["variable_step"] > 0, 1)
        rate, ipc_n, secs = (rate1, ipc, secs1)
        if nt > 1:
            rate, ipc_n, secs = cpu_baseline(dump, args.cpu_steps, cfg["q"], cfg["route_step"],
                                             cfg["variable_step"] > 0, nt)
        os.remove(dump)
        try:
            ref = ref_baseline(nt)
        except Exception as exc:        # noqa: BLE001 -- a baseline, never the measurement
            ref = {"error": repr(exc)}
        cpu = {"value": round(rate, 1), "unit": "link-updates/s", "cores": nt, "kind": "port",
               "reference": ref,
               "cpu_model": cpu_model(),
               "single_thread": {"value": round(rate1, 1), "cores": 1, "seconds": round(secs1, 2)},
               "sample": "%d routing steps (%.1f s on %d threads, %.2f iterations/step) of the same "
                         "%dx%d grid continuing from the GPU run's state after the timed window; "
                         "oracle/dw_oracle.c with its per-link and per-node loops on OpenMP "
                         "threads (node sums serial, as the reference)"
                         % (args.cpu_steps, secs, nt, ipc_n, cfg["grid"], cfg["grid"])}

    if rank == 0:
        value = updates / elapsed
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "link-updates/s",
            # value counts every conduit in every Picard iteration that ran
            # (SURVEY 8d); conduits bypassed by findBypassedLinks count too.
            # effective_value counts only the conduits actually updated (the
            # bypass fraction measured over the timing-mode steps)
            "effective_value": None if eff is None else round(value * eff, 1),
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic",
            "config": {"workload": workload,
                       "conduits": nL, "nodes": nN, "pollutants": cfg["pollutants"],
                       "spinup_steps": cfg["spinup"],
                       "iterations_per_step": round(iters / args.steps, 3),
                       "nonconverged_steps": nonconv,
                       "surcharged_pct": round(surcharged, 2),
                       # step graphs the timed steps launched (Router::step's per-step choice)
                       "step_graphs": {g: c1["steps_" + g] - c0["steps_" + g]
                                       for g in ("unrolled", "tail", "sparse", "list")},
                       "sim_time_at_end_s": round(t_days * 86400.0, 1),
                       "parallelism": ("link-partitioned x%d (node blocks: see partition); per Picard iteration "
                                       "%s of the neighbours' ghost-link values and an "
                                       "all-reduce(max) of the convergence flag"
                                       % (world, {"ipc": "device stores into the peers' memory (IPC)",
                                                  "rccl": "RCCL ncclSend/ncclRecv"}.get(
                                                      transport.split()[0], "host-transport (gloo) exchange"))
                                       )
                                      if world > 1 else
                                      ("single rank through the partitioned RCCL path (captured ncclSend/"
                                       "ncclRecv and flag all-reduce every Picard iteration)"
                                       if args.rccl_1rank else "single"),
                       "backend": backend,
                       "transport": transport,
                       "partition": None if world == 1 else (
                           ("blocks of %s nodes dealt to the ranks in turn (SWMM5_PART_BLOCK)"
                            % os.environ["SWMM5_PART_BLOCK"]) if int(os.environ.get("SWMM5_PART_BLOCK", "0")) > 0 else
                           "contiguous row strips of equal node count" if balance is None else
                           ("two regions of equal weight 1 + %.3f x measured sparse updates per node and step: "
                            "the surcharged band (weight excess at least a quarter of the largest) in 2R blocks "
                            "dealt 0..R-1, R-1..0, and the rest in R blocks (%s)" % (balance["lambda"], balance["source"]))
                           if args.balance == "auto" else
                           "contiguous node blocks of equal weight: 1 + %.3f x measured sparse node updates per "
                           "step (%s)" % (balance["lambda"], balance["source"]))},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
