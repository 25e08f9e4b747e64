"""Worker process for tests/test_multigpu.py (test infrastructure).

Runs the engine on one rank of a partitioned network.  Transport:
  host  -- swmmx_setExchange with a gloo all-reduce callback (works with all
           ranks on one GPU, which RCCL refuses)
  rccl  -- RCCL (one rank only on a one-GPU box: exercises the captured
           ncclSend / ncclRecv and flag all-reduce path)
Writes the owned part of the final state to an .npz (and, with
WORKER_SAVE=1, the binary results file next to it, rank 0 only).

With WORKER_OUT0=<path>, rank 0 writes its binary results there instead
(e.g. /dev/full: every write fails) and the worker expects an error: it runs
start / steps / end, writes the error codes each returned (and the message)
to the .npz and exits 0 when some call failed.

usage: python _mgpu_worker.py INP STEPS OUT.npz TRANSPORT     (env: RANK, WORLD_SIZE, MASTER_*)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "stormwater-management-model_amd"))

import swmm5  # noqa: E402


def main():
    inp, steps, out, transport = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    s = swmm5.SWMM()
    if transport in ("host", "ipc"):
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)

        def xchg(arr, op):
            t = torch.from_numpy(arr)
            dist.all_reduce(t, op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MIN)

        s.set_partition(rank, world)
        s.set_exchange(xchg)
        ww = os.environ.get("WORKER_WEIGHTS", "")
        if ww == "ramp":                 # a weighted partition: later nodes weigh up to 4x
            nN = int(os.environ["WORKER_NODES"])
            s.set_partition_weights(np.linspace(1.0, 4.0, nN))
        elif ww.startswith("file:"):     # weights saved by the test (e.g. bench.py's calibrated ones)
            s.set_partition_weights(np.load(ww[5:]))
        if ww and os.environ.get("WORKER_PARTMODE"):   # e.g. two_region: the band and the rest dealt separately
            s.set_partition_mode(os.environ["WORKER_PARTMODE"])
        if transport == "ipc":          # device stores into the peers' memory; gloo bootstraps it
            s.set_transport("ipc")
    else:
        assert world == 1
        s.set_partition(0, 1, s.nccl_unique_id())
    tag = os.path.splitext(out)[0]      # <out>.rpt / <out>.out: one pair per run and rank
    out0 = os.environ.get("WORKER_OUT0")
    if out0:                            # an error is expected: report which call failed, on every rank
        assert s.open(inp, tag + ".rpt", out0 if rank == 0 else tag + ".out") == 0, s.getError()
        codes = [s.start(True), 0, 0]
        if codes[0] == 0:
            codes[1] = s.run_steps(steps)[0]
            codes[2] = s.end()
        msg = s.getError()
        s.close()
        np.savez(out, codes=np.array(codes), msg=np.frombuffer(str(msg).encode(), dtype=np.uint8))
        if transport in ("host", "ipc"):
            import torch.distributed as dist
            dist.destroy_process_group()
        sys.exit(0 if any(codes) else 3)
    assert s.open(inp, tag + ".rpt", tag + ".out") == 0, s.getError()
    # WORKER_SAVE=1: swmm_start(1), the binary results file (rank 0 writes it)
    assert s.start(os.environ.get("WORKER_SAVE") == "1") == 0, s.getError()
    err, _ = s.run_steps(steps)
    assert err == 0, s.getError()
    c = s.counters()
    res = {
        "node_owner": s.owners(swmm5.NODE),
        "link_owner": s.owners(swmm5.LINK),
        "counters": np.array([c["steps"], c["iterations"], c["nonconverged"]]),
        "graphs": np.array([c["steps_unrolled"], c["steps_list"]]),
        "transport": np.frombuffer(s.transport().encode(), dtype=np.uint8),
    }
    for f in ("newDepth", "newVolume", "inflow", "outflow", "overflow"):
        res["node." + f] = s.get_array("node." + f)
    for f in ("newFlow", "newDepth", "newVolume", "froude", "a1", "q1", "dqdh", "surfArea1", "surfArea2"):
        res["link." + f] = s.get_array("link." + f)
    nN, nL = s.getCount(swmm5.NODE), s.getCount(swmm5.LINK)
    P = s.get_array("node.newQual").size // max(nN, 1)
    for q in range(P):                  # pollutant concentrations, one array per pollutant
        res["node.qual%d" % q] = s.get_array("node.newQual").reshape(P, nN)[q].copy()
        res["link.qual%d" % q] = s.get_array("link.newQual").reshape(P, nL)[q].copy()
    s.end()
    _, ferr, _ = s.getMassBalErr()
    res["flow_error"] = np.array([ferr])
    s.close()
    np.savez(out, **res)
    if transport in ("host", "ipc"):
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
