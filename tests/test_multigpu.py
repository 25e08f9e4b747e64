"""Multi-GPU partitioned routing (include/swmm5_mi355x.h).

CPU (no GPU needed):
  * owner rules of the partition (node blocks, conduit -> node1's rank,
    outfall -> its conduit's rank) checked against a numpy restatement;
  * the engine's own ghost-link layout (swmmx_getPartition) for 2, 3 and 8
    ranks, row strips and node blocks dealt in turn: every held node's
    incidence row holds exactly its links in global order, every ghost is
    sent by its owner in the receiver's order;
  * a world_size-2 gloo job of the neighbour exchange on that layout: each
    rank packs the links it sends (sendLink), exchanges them with its
    neighbours (gloo send / recv), unpacks them into its ghost slots and sums
    every held node over its row -- bitwise the whole network's serial sums.
GPU:
  * 2 and 3 ranks on the one GPU with the host (gloo) transport against the
    same network on one GPU: owned node / link state BITWISE equal, same
    iteration and non-convergence counts (fixed step; surcharged variable
    step; 3 pollutants; pumps and regulators; the list graph on every step,
    with strips, interleaved blocks, pollutants and regulators);
  * results and hot-start files byte-identical to one GPU's; a write error on
    rank 0 stops every rank; SKIP_STEADY_STATE with two ranks bitwise equal
    to one GPU (its .out byte-identical);
  * the IPC transport (device stores into the peers' memory, captured step
    graphs): the same bitwise cases with 2 and 3 ranks on the one GPU, and a
    rank that stops answering makes every rank fail within the deadline;
  * 1 rank through the RCCL path (captured ncclSend/ncclRecv + flag
    all-reduce): bitwise equal to the single-GPU engine;
  * the 4M-conduit configs[4] network split in two strips, bitwise.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import netgen
import swmm5

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "_mgpu_worker.py")


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _grid(tmp_path, nx=24, ny=20, **kw):
    inp = str(tmp_path / "g.inp")
    kw.setdefault("end_time", "02:00:00")
    netgen.write_grid(inp, nx, ny, **kw)
    return inp


def _topology(inp, tmp_path):
    s = swmm5.SWMM()
    assert s.open(inp, str(tmp_path / "t.rpt"), str(tmp_path / "t.out")) == 0
    assert s.start_host() == 0
    dump = str(tmp_path / "t.bin")
    s.export_state(dump)
    s.close()
    from _dumpio import read_dump
    return read_dump(dump)


def _owners(inp, tmp_path, rank, world):
    s = swmm5.SWMM()
    s.set_partition(rank, world)
    try:
        assert s.open(inp, str(tmp_path / "o.rpt"), str(tmp_path / "o.out")) == 0
        return s.owners(swmm5.NODE), s.owners(swmm5.LINK)
    finally:
        s.close()
        s.set_partition(0, 1)


def _ref_owners(n1, n2, ntype, nN, world):
    node = (np.arange(nN, dtype=np.int64) * world // nN).astype(np.int32)
    link = node[n1].copy()
    OUTFALL = 1
    for j in range(len(n1)):
        if ntype[n2[j]] == OUTFALL:
            node[n2[j]] = link[j]
        elif ntype[n1[j]] == OUTFALL:
            node[n1[j]] = link[j]
    return node, link


@pytest.mark.parametrize("world", [2, 3, 8])
def test_partition_owner_rules(world, tmp_path):
    inp = _grid(tmp_path)
    d = _topology(inp, tmp_path)
    n1, n2 = d["link.node1"].astype(int), d["link.node2"].astype(int)
    ntype = d["node.type"].astype(int)
    ref_node, ref_link = _ref_owners(n1, n2, ntype, len(ntype), world)
    for rank in (0, world - 1):
        node, link = _owners(inp, tmp_path, rank, world)
        np.testing.assert_array_equal(node, ref_node)
        np.testing.assert_array_equal(link, ref_link)
    # every rank owns a contiguous strip of rows and about 1/world of the conduits
    counts = np.bincount(ref_link, minlength=world)
    assert counts.min() > 0.5 * len(n1) / world


def _layout(inp, tmp_path, rank, world):
    """The engine's partition of `inp` as seen by `rank` (host-only open)."""
    s = swmm5.SWMM()
    s.set_partition(rank, world)
    try:
        assert s.open(inp, str(tmp_path / "p.rpt"), str(tmp_path / "p.out")) == 0
        return {k: s.partition_array(k) for k in ("lnode", "llink", "lghost", "nbr", "sendOff",
                                                   "sendLink", "recvOff", "rowptr", "csr", "hasGhost")}
    finally:
        s.close()
        s.set_partition(0, 1)


def test_weighted_partition_layout(tmp_path):
    """swmmx_setPartitionWeights: contiguous node blocks of equal total
    weight (node i to the rank whose share holds the midpoint of its weight
    interval); every held node still sees all its conduits in global order
    and every ghost is sent by its owner in the receiver's order."""
    inp = _grid(tmp_path, 24, 20)
    d = _topology(inp, tmp_path)
    n1, n2 = d["link.node1"].astype(int), d["link.node2"].astype(int)
    nN = len(d["node.type"])
    w = np.linspace(1.0, 4.0, nN)
    for world in (2, 3):
        mid = np.cumsum(w) - 0.5 * w
        ref = np.minimum((mid * world / w.sum()).astype(int), world - 1)
        lays = []
        for r in range(world):
            s = swmm5.SWMM()
            s.set_partition(r, world)
            s.set_partition_weights(w)
            try:
                assert s.open(inp, str(tmp_path / "w.rpt"), str(tmp_path / "w.out")) == 0
                owner = s.owners(swmm5.NODE)
                lays.append({k: s.partition_array(k) for k in ("lnode", "llink", "lghost", "nbr", "sendOff",
                                                               "sendLink", "recvOff", "rowptr", "csr")})
            finally:
                s.close()
                s.set_partition(0, 1)
            junction = d["node.type"].astype(int) != 1
            np.testing.assert_array_equal(owner[junction], ref[junction])
        counts = np.bincount(owner[:-1], minlength=world)
        assert counts[0] > counts[-1]                      # the heavier tail is split finer
        rows = _incident(n1, n2, nN)
        for r, L in enumerate(lays):
            loc = np.concatenate([L["llink"], L["lghost"]])
            rp, csr = L["rowptr"], L["csr"]
            for i, g in enumerate(L["lnode"]):
                got = [(int(loc[e & 0x7FFFFFFF]), int((e >> 31) & 1)) for e in csr[rp[i]:rp[i + 1]]]
                assert got == rows[g], (r, g)
            for k, s_ in enumerate(L["nbr"]):
                S = lays[s_]
                ks = list(S["nbr"]).index(r)
                np.testing.assert_array_equal(L["lghost"][L["recvOff"][k]:L["recvOff"][k + 1]],
                                              S["llink"][S["sendLink"][S["sendOff"][ks]:S["sendOff"][ks + 1]]])


def test_two_region_partition_layout(tmp_path):
    """swmmx_setPartitionMode(1): the hot nodes (weight excess at least a quarter of
    the largest: here the last four grid rows, a surcharged band) are cut into
    2 x ranks contiguous blocks of equal weight dealt 0, 1, .., 1, 0, the
    others into one block per rank -- every rank owns an equal share of the
    band and of the rest; the layout keeps every held node's conduits in
    global order."""
    inp = _grid(tmp_path, 24, 20)
    d = _topology(inp, tmp_path)
    n1, n2 = d["link.node1"].astype(int), d["link.node2"].astype(int)
    nN = len(d["node.type"])
    junction = d["node.type"].astype(int) != 1
    w = np.ones(nN)
    band = np.arange(nN) >= nN - 1 - 4 * 20          # the last four rows (and the outfall)
    w[band] = 7.0
    w[band & (np.arange(nN) % 3 == 0)] = 6.0         # uneven inside the band: still >= the cut (4.0)
    rows = _incident(n1, n2, nN)
    for world in (2, 3):
        lays, owner = [], None
        for r in range(world):
            s = swmm5.SWMM()
            s.set_partition(r, world)
            s.set_partition_weights(w)
            assert s.set_partition_mode("two_region") == 0
            try:
                assert s.open(inp, str(tmp_path / "w.rpt"), str(tmp_path / "w.out")) == 0
                owner = s.owners(swmm5.NODE)
                lays.append({k: s.partition_array(k) for k in ("lnode", "llink", "lghost", "rowptr", "csr")})
            finally:
                s.close()
                s.set_partition_mode("contiguous")
                s.set_partition_weights(None)
                s.set_partition(0, 1)
        # reference: the band in 2 x world equal-weight blocks dealt
        # 0, 1, .., world-1, world-1, .., 0; the rest in world blocks
        ref = np.zeros(nN, dtype=int)
        for sel, nb in ((band, 2 * world), (~band, world)):
            idx = np.nonzero(sel)[0]
            ww = w[idx]
            mid = np.cumsum(ww) - 0.5 * ww
            b = np.minimum((mid * nb / ww.sum()).astype(int), nb - 1)
            ref[idx] = np.where(b < world, b, 2 * world - 1 - b) if nb == 2 * world else b
        np.testing.assert_array_equal(owner[junction], ref[junction])
        hot = np.bincount(owner[band & junction], minlength=world)
        cold = np.bincount(owner[~band & junction], minlength=world)
        assert hot.max() - hot.min() <= 2 and cold.max() - cold.min() <= 2, (hot, cold)
        for r, L in enumerate(lays):
            loc = np.concatenate([L["llink"], L["lghost"]])
            rp, csr = L["rowptr"], L["csr"]
            for i, g in enumerate(L["lnode"]):
                got = [(int(loc[e & 0x7FFFFFFF]), int((e >> 31) & 1)) for e in csr[rp[i]:rp[i + 1]]]
                assert got == rows[g], (r, g)


def _incident(n1, n2, nN):
    rows = [[] for _ in range(nN)]
    for j in range(len(n1)):
        rows[n1[j]].append((j, 0))
        rows[n2[j]].append((j, 1))
    return rows


@pytest.mark.parametrize("world,block", [(2, 0), (3, 0), (8, 0), (2, 40), (3, 24), (8, 20)])
def test_partition_ghost_layout(world, block, tmp_path, monkeypatch):
    """Every rank's held nodes see all their conduits -- owned ones and ghosts
    -- in ascending global order (the reference's summation order), and what
    each owner sends is exactly what the receiver expects, in its order.  For
    contiguous strips (block 0) and for node blocks dealt to the ranks in turn
    (SWMM5_PART_BLOCK: node i, unless an outfall, goes to rank
    (i // block) % world)."""
    monkeypatch.setenv("SWMM5_PART_BLOCK", str(block))
    inp = _grid(tmp_path, 24, 20)
    d = _topology(inp, tmp_path)
    n1, n2 = d["link.node1"].astype(int), d["link.node2"].astype(int)
    nN = len(d["node.type"])
    rows = _incident(n1, n2, nN)
    node_owner, link_owner = _owners(inp, tmp_path, 0, world)
    if block:
        junction = d["node.type"].astype(int) != 1
        idx = np.arange(nN)[junction]
        np.testing.assert_array_equal(node_owner[junction], (idx // block) % world)
        np.testing.assert_array_equal(link_owner, node_owner[n1])
    lay = [_layout(inp, tmp_path, r, world) for r in range(world)]
    for r, L in enumerate(lay):
        loc = np.concatenate([L["llink"], L["lghost"]])          # local -> global link
        assert (link_owner[L["llink"]] == r).all() and (link_owner[L["lghost"]] != r).all()
        rp, csr = L["rowptr"], L["csr"]
        for i, g in enumerate(L["lnode"]):
            ent = csr[rp[i]:rp[i + 1]]
            got = [(int(loc[e & 0x7FFFFFFF]), int((e >> 31) & 1)) for e in ent]
            assert got == rows[g], (r, g, got, rows[g])
            assert bool(L["hasGhost"][i]) == any(link_owner[j] != r for j, _ in rows[g])
        # ghosts from each neighbour == what that neighbour sends to r
        for k, s_ in enumerate(L["nbr"]):
            ghosts = L["lghost"][L["recvOff"][k]:L["recvOff"][k + 1]]
            S = lay[s_]
            ks = list(S["nbr"]).index(r)
            sent = S["llink"][S["sendLink"][S["sendOff"][ks]:S["sendOff"][ks + 1]]]
            np.testing.assert_array_equal(ghosts, sent)
        assert len(L["lghost"]) == L["recvOff"][-1]
    if world > 2 and not block:        # strips: only adjacent ranks exchange
        for r, L in enumerate(lay):
            assert set(L["nbr"]) <= {r - 1, r + 1}, (r, L["nbr"])


def _node_sums(q, lat, rp, csr, nodes):
    """k_node's gather (dynwave.c:528-589): lateral inflow, then each link of
    the node's row in order"""
    inflow = np.zeros(len(nodes))
    outflow = np.zeros(len(nodes))
    for i in range(len(nodes)):
        a = lat[i]
        fin, fout = (a, 0.0) if a >= 0.0 else (0.0, -a)
        for e in csr[rp[i]:rp[i + 1]]:
            f = q[e & 0x7FFFFFFF]
            if (e >> 31) & 1 == 0:
                if f >= 0.0:
                    fout += f
                else:
                    fin -= f
            else:
                if f >= 0.0:
                    fin += f
                else:
                    fout -= f
        inflow[i], outflow[i] = fin, fout
    return inflow, outflow


def _exchange_worker(rank, world, port, L, qg, latg, outq):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nown = len(L["llink"])
    q = np.zeros(nown + len(L["lghost"]))
    q[:nown] = qg[L["llink"]]                                   # this rank's own links
    send = torch.from_numpy(q[L["sendLink"]].copy())            # k_xpack
    recv = torch.zeros(len(L["lghost"]), dtype=torch.float64)
    reqs = []
    for k, nb in enumerate(L["nbr"]):                           # neighbour send / recv
        a, b = L["sendOff"][k], L["sendOff"][k + 1]
        if b > a:
            reqs.append(dist.isend(send[a:b].contiguous(), int(nb)))
        a, b = L["recvOff"][k], L["recvOff"][k + 1]
        if b > a:
            buf = torch.zeros(b - a, dtype=torch.float64)
            reqs.append((dist.irecv(buf, int(nb)), a, buf))
    for r in reqs:
        if isinstance(r, tuple):
            r[0].wait()
            recv[r[1]:r[1] + len(r[2])] = r[2]
        else:
            r.wait()
    q[nown:] = recv.numpy()                                     # k_xunpack
    inflow, outflow = _node_sums(q, latg[L["lnode"]], L["rowptr"], L["csr"], L["lnode"])
    outq.put((rank, inflow, outflow))
    dist.barrier()
    dist.destroy_process_group()


def test_neighbour_exchange_gloo_world2(tmp_path):
    """The neighbour exchange on the engine's own layout as a world-size-2
    gloo job: every held node's sums -- owned nodes and replicas alike -- are
    bitwise the whole network's serial link-order sums.  (The device side,
    k_xpack / k_xunpack / k_node, runs in the GPU tests below.)"""
    import torch.multiprocessing as mp
    inp = _grid(tmp_path)
    d = _topology(inp, tmp_path)
    n1, n2 = d["link.node1"].astype(int), d["link.node2"].astype(int)
    nN, nL = len(d["node.type"]), len(n1)
    rng = np.random.default_rng(20250215)
    q = rng.normal(0.0, 1.0, nL)
    q[::7] = 0.0
    lat = np.abs(rng.normal(0.0, 0.1, nN))
    world = 2
    lay = [_layout(inp, tmp_path, r, world) for r in range(world)]
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, lay[r], q, lat, outq))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, fin, fout = outq.get(timeout=120)
        res[r] = (fin, fout)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # whole-network sums (serial scatter, link order: dynwave.c:398-411)
    inflow = np.where(lat >= 0, lat, 0.0)
    outflow = np.where(lat < 0, -lat, 0.0)
    for j in range(nL):
        a, b, f = n1[j], n2[j], q[j]
        if f >= 0:
            outflow[a] += f
            inflow[b] += f
        else:
            inflow[a] -= f
            outflow[b] -= f
    held = np.zeros(nN, dtype=int)
    for r in range(world):
        nodes = lay[r]["lnode"]
        held[nodes] += 1
        np.testing.assert_array_equal(res[r][0], inflow[nodes])
        np.testing.assert_array_equal(res[r][1], outflow[nodes])
    assert (held >= 1).all() and (held == 2).sum() > 0            # replicas exist and agree


def test_partition_keeps_regulator_nodes_on_one_rank(tmp_path):
    """Pumps and regulators (k_nc: link-order running totals of their end
    nodes) keep their end nodes and every link touching them on one rank."""
    import _golden
    inp = _golden.inp("example_regulators")
    d = _topology(inp, tmp_path)
    ltype = d["link.type"].astype(int)
    n1, n2 = d["link.node1"].astype(int), d["link.node2"].astype(int)
    for world in (2, 3):
        node_owner, link_owner = _owners(inp, tmp_path, 0, world)
        deferred = set(n1[ltype != 0]) | set(n2[ltype != 0])
        for j in range(len(n1)):
            for n in (n1[j], n2[j]):
                if n in deferred:
                    assert link_owner[j] == node_owner[n], (world, j, n)
        lay = [_layout(inp, tmp_path, r, world) for r in range(world)]
        for n in deferred:
            assert sum(int(n in set(L["lnode"])) for L in lay) == 1, (world, n)


def _run_workers(inp, steps, tmp_path, world, transport, tag, save=False, extra_env=None, timeout=600):
    port = _free_port()
    procs = []
    outs = []
    for r in range(world):
        out = str(tmp_path / ("%s_r%d.npz" % (tag, r)))
        outs.append(out)
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORKER_SAVE="1" if save else "0",
                   **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, WORKER, inp, str(steps), out, transport],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    try:
        for p in procs:
            o, _ = p.communicate(timeout=timeout)
            assert p.returncode == 0, o.decode()[-3000:]
    finally:
        for p in procs:                 # a hung rank must not outlive the test
            if p.poll() is None:
                p.kill()
                p.wait()
    return [dict(np.load(o)) for o in outs]


def _merge(parts):
    node = {k: np.zeros_like(v) for k, v in parts[0].items() if k.startswith("node.")}
    link = {k: np.zeros_like(v) for k, v in parts[0].items() if k.startswith("link.")}
    for r, part in enumerate(parts):
        nm = part["node_owner"] == r
        lm = part["link_owner"] == r
        for k in node:
            node[k][nm] = part[k][nm]
        for k in link:
            link[k][lm] = part[k][lm]
    return node, link


def _assert_bitwise(parts, one):
    node, link = _merge(parts)
    for k, v in list(node.items()) + list(link.items()):
        np.testing.assert_array_equal(v, one[k], err_msg=k)
    for part in parts:
        np.testing.assert_array_equal(part["counters"], one["counters"])
        assert abs(part["flow_error"][0] - one["flow_error"][0]) < 1e-3


def _transport_of(part):
    return bytes(part["transport"]).decode()


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["host", "ipc"])
@pytest.mark.parametrize("kw,steps,surcharged,world", [
    (dict(route_step=1.0), 120, False, 2),
    # the benchmark's regime: surcharged, non-converging, iterations >= 2 with
    # bypassed conduits on every rank and the cross-rank convergence flag
    (dict(route_step=5.0, variable_step=0.75, diameter=1.0, q=0.5), 250, True, 2),
    # three strips: ranks 0 and 2 share no node, so a node left unconverged
    # between ranks 1 and 2 must still keep rank 0 iterating
    (dict(route_step=5.0, variable_step=0.75, diameter=1.0, q=0.5), 250, True, 3),
    # water quality (qualrout): ghost links' concentrations move once per step
    (dict(route_step=5.0, variable_step=0.75, diameter=1.0, q=0.5, pollutants=3), 250, True, 2)])
def test_ranks_match_one_gpu_bitwise(kw, steps, surcharged, world, transport, tmp_path):
    """Every held node is summed over all its links in the reference's order
    on every rank (ghost links exchanged between neighbours), so the
    partitioned run is bitwise equal to one GPU.  host: gloo through the
    host, eager launches; ipc: the captured step graphs with the ghost
    values, convergence flags and Courant limits stored by each rank's
    kernels straight into its peers' memory (the ranks share this box's
    GPU: IPC within one device)."""
    inp = _grid(tmp_path, 30, 30, **kw)
    one = _run_workers(inp, steps, tmp_path, 1, "host", "one")[0]
    if surcharged:
        st, its, nonconv = one["counters"]
        assert nonconv > 10 and its / st > 2.5, one["counters"]
        assert (one["node.newDepth"][:-1] > kw["diameter"]).sum() > 100
    parts = _run_workers(inp, steps, tmp_path, world, transport, "part")
    for part in parts:
        assert _transport_of(part) == transport, _transport_of(part)
    _assert_bitwise(parts, one)
    if kw.get("pollutants"):
        assert (one["node.qual2"] > 1.0).mean() > 0.5


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_ipc_stalled_rank_fails_every_rank(world, tmp_path):
    """Failure detection on the exchange path (swmm5.c:420's sticky error
    contract): the last rank stops posting its ghost values and flags at step
    20 (test hook SWMM5_XCHG_STALL); the others' bounded waits (3 s,
    SWMM5_XCHG_TIMEOUT) give up, tell every rank to stop, and every rank's
    swmm_step returns error 500 -- no rank hangs."""
    import time
    inp = _grid(tmp_path, 30, 30, route_step=5.0, variable_step=0.75, diameter=1.0, q=0.5)
    t0 = time.time()
    parts = _run_workers(inp, 400, tmp_path, world, "ipc", "stall",
                         extra_env={"WORKER_OUT0": str(tmp_path / "stall0.out"),
                                    "SWMM5_XCHG_STALL": "%d:20" % (world - 1), "SWMM5_XCHG_TIMEOUT": "3"},
                         timeout=240)
    elapsed = time.time() - t0
    for p in parts:
        codes = [int(c) for c in p["codes"]]
        msg = bytes(p["msg"]).decode()
        assert codes[0] == 0 and codes[1] == 500, (codes, msg)
        assert "exchange" in msg, msg
    assert elapsed < 150, elapsed


def _grid_with_regulators(tmp_path, n=20):
    """An n x n grid (variable step) in which three conduits become a side
    orifice (upper strip), a transverse weir across the middle (the two-rank
    strip boundary) and a functional outlet (lower strip)."""
    import re
    inp = _grid(tmp_path, n, n, route_step=5.0, variable_step=0.75, diameter=1.0, q=0.08)
    text = open(inp).read()
    head, rest = text.split("[CONDUITS]", 1)
    cond, rest = rest.split("[XSECTIONS]", 1)
    xs, tail = rest.split("\n\n", 1)

    def pick(row_from, row_to):
        for line in cond.splitlines():
            m = re.match(r"(C\d+)\s+J(\d+)_(\d+)\s+J(\d+)_(\d+)", line)
            if m and int(m.group(2)) == row_from and int(m.group(4)) == row_to and 2 <= int(m.group(3)) < n - 2:
                return line.split()
        raise AssertionError((row_from, row_to))
    ori, weir, outl = pick(3, 4), pick(n // 2 - 1, n // 2), pick(3 * n // 4, 3 * n // 4 + 1)
    drop = {ori[0], weir[0], outl[0]}
    keep = lambda block: "\n".join(l for l in block.splitlines() if not (l.split() and l.split()[0] in drop))
    out = head + "[CONDUITS]" + keep(cond) + "[XSECTIONS]" + keep(xs) + "\n"
    out += "%s CIRCULAR 1.0 0 0 0\n%s RECT_OPEN 1.0 3.0 0 0\n\n" % (ori[0], weir[0])
    out += "[ORIFICES]\n%s %s %s SIDE 0.0 0.65 NO\n\n" % (ori[0], ori[1], ori[2])
    out += "[WEIRS]\n%s %s %s TRANSVERSE 0.1 3.33 NO 0 0 YES\n\n" % (weir[0], weir[1], weir[2])
    out += "[OUTLETS]\n%s %s %s 0.0 FUNCTIONAL/DEPTH 2.0 0.5 NO\n\n" % (outl[0], outl[1], outl[2])
    out += tail
    path = str(tmp_path / "greg.inp")
    open(path, "w").write(out)
    return path


@pytest.mark.gpu
@pytest.mark.parametrize("world,block,pollutants,transport", [
    (2, 0, 0, "host"), (3, 0, 0, "host"), (2, 90, 0, "host"), (3, 60, 0, "host"), (2, 0, 2, "host"),
    (2, 0, 0, "ipc"), (3, 60, 0, "ipc"), (2, 0, 2, "ipc"), (3, -1, 0, "ipc"), (3, -2, 0, "ipc"),
    (2, 0, 2, "ipc_fused"), (3, -2, 0, "ipc_fused")])
def test_ranks_list_graph_bitwise(world, block, pollutants, transport, tmp_path):
    """The list graph (iterations k >= 2 as unconverged-list walks and
    live-list node passes, each followed by the neighbour exchange and the
    flag all-reduce) on several ranks: every step runs it and the run is
    bitwise equal to one GPU's (which runs it too) -- the surcharged,
    non-converging 30 x 30 grid, host transport; with row strips and with
    node blocks dealt to the ranks in turn (SWMM5_PART_BLOCK: 3 and 2 grid
    rows per block, every rank holding part of the surcharged corner); with
    node weights (contiguous blocks of equal weight, and two regions each cut
    into equal-weight blocks: every rank holds two separate stretches); and
    with two pollutants (the frozen junctions' final depths then come from the
    quality kernel, after the ghost links' concentrations moved); the IPC
    cases also with the one-launch exchange (k_ipc_xchg)."""
    inp = _grid(tmp_path, 30, 30, route_step=5.0, variable_step=0.75, diameter=1.0, q=0.5, pollutants=pollutants)
    env = {"SWMM5_SPARSE": "3", "SWMM5_PART_BLOCK": str(max(block, 0))}
    if block < 0:                         # a weighted partition (node weights 1 .. 4, swmmx_setPartitionWeights)
        env.update(WORKER_WEIGHTS="ramp", WORKER_NODES=str(30 * 30 + 1))
    if block == -2:                       # two regions: the heavier half and the rest, each cut in three
        env.update(WORKER_PARTMODE="two_region")
    one = _run_workers(inp, 250, tmp_path, 1, "host", "one", extra_env=env)[0]
    st, its, nonconv = one["counters"]
    assert nonconv > 10 and its / st > 2.5, one["counters"]
    if transport == "ipc_fused":          # the one-launch exchange (chosen when every rank has its own GPU)
        env["SWMM5_XCHG_FUSED"] = "1"
        transport = "ipc"
    parts = _run_workers(inp, 250, tmp_path, world, transport, "part", extra_env=env)
    for part in parts:
        assert part["graphs"][1] == part["counters"][0], (part["graphs"], part["counters"])
        assert _transport_of(part) == transport
    _assert_bitwise(parts, one)


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["host", "ipc"])
def test_eight_ranks_bitwise_benchmark_regime(transport, tmp_path):
    """Eight ranks (the driver's node size) on this box's one GPU, in the
    benchmark's regime: a surcharged, non-converging 100 x 100 grid (SURVEY
    section 6's q = 0.1 row) in eight row strips, every step on the list graph,
    shared nodes freezing.  The surcharged region spans several strips, so
    iterations k >= 2 have live lists on several ranks; every owned node and
    link field is bitwise the one-GPU run's, with equal iteration and
    non-convergence counts."""
    inp = _grid(tmp_path, 100, 100, route_step=5.0, variable_step=0.75, diameter=1.0, q=0.1, end_time="00:40:00")
    env = {"SWMM5_SPARSE": "3"}
    one = _run_workers(inp, 100000, tmp_path, 1, "host", "one", extra_env=env)[0]
    st, its, nonconv = one["counters"]
    assert nonconv > 10 and its / st > 2.5, one["counters"]
    parts = _run_workers(inp, 100000, tmp_path, 8, transport, "eight", extra_env=env, timeout=900)
    for part in parts:
        assert part["graphs"][1] == part["counters"][0], (part["graphs"], part["counters"])
        assert _transport_of(part) == transport
    owner = parts[0]["node_owner"]
    sur = one["node.newDepth"][:-1] > 1.0
    ranks_surcharged = sorted(set(owner[:-1][sur].tolist()))
    assert len(ranks_surcharged) >= 3, ranks_surcharged       # live sparse work on several ranks
    _assert_bitwise(parts, one)


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", ["0", "3"])
def test_regulators_two_ranks_bitwise(sparse, tmp_path):
    """An orifice, a weir across the strip boundary and an outlet (k_nc) with
    two ranks: each regulator's end nodes and the links touching them stay on
    one rank, every other node is exchanged as usual; bitwise equal to one
    GPU.  With the unrolled graph, and with the list graph on every step
    (k_nc after each k_node_list), whose one-GPU run is bitwise equal to the
    unrolled one's too."""
    inp = _grid_with_regulators(tmp_path)
    env = {"SWMM5_SPARSE": sparse}
    one = _run_workers(inp, 300, tmp_path, 1, "host", "one", extra_env=env)[0]
    parts = _run_workers(inp, 300, tmp_path, 2, "host", "two", extra_env=env)
    assert all((p["link_owner"] == r).any() for r, p in enumerate(parts))
    _assert_bitwise(parts, one)
    if sparse == "3":
        for run in [one] + parts:
            assert run["graphs"][1] == run["counters"][0], (run["graphs"], run["counters"])
        unrolled = _run_workers(inp, 300, tmp_path, 1, "host", "unrolled", extra_env={"SWMM5_SPARSE": "0"})[0]
        assert unrolled["graphs"][1] == 0, unrolled["graphs"]
        _assert_bitwise([unrolled], one)


@pytest.mark.gpu
@pytest.mark.parametrize("world,pollutants", [(2, 0), (3, 2)])
def test_ranks_write_one_gpu_results_and_hotstart(world, pollutants, tmp_path):
    """swmm_start(1) and SAVE HOTSTART with several ranks (output.c:457-695,
    hotstart.c:224-262): the owners' packed period results are gathered to
    rank 0, which writes the binary results file, and the final state's hot
    start fields likewise.  Both files are byte-identical to the one-GPU
    run's (surcharged, variable-step 30 x 30 grid, every object reported, a
    period every minute); the other ranks write no results file."""
    kw = dict(route_step=5.0, variable_step=0.75, diameter=1.0, q=0.5, pollutants=pollutants,
              report_step="00:01:00", report_all=True)
    runs = {}
    for name, w in (("one", 1), ("many", world)):
        hs = str(tmp_path / ("%s.hsf" % name))
        inp = str(tmp_path / ("%s.inp" % name))
        netgen.write_grid(inp, 30, 30, end_time="00:20:00", files='SAVE HOTSTART "%s"' % hs, **kw)
        parts = _run_workers(inp, 100000, tmp_path, w, "host", name, save=True)
        runs[name] = (parts, hs, str(tmp_path / ("%s_r0.out" % name)))
    one_out = open(runs["one"][2], "rb").read()
    many_out = open(runs["many"][2], "rb").read()
    assert len(one_out) > 30 * 30 * 6 * 4 * 10            # ten or more reporting periods
    assert many_out == one_out
    assert open(runs["many"][1], "rb").read() == open(runs["one"][1], "rb").read()
    for r in range(1, world):
        assert not os.path.exists(str(tmp_path / ("many_r%d.out" % r)))
    st, its, nonconv = runs["one"][0][0]["counters"]
    assert nonconv > 0 and its / st > 2.5, (st, its, nonconv)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [30, 6])
def test_rank0_write_error_stops_every_rank(n, tmp_path):
    """Rank 0 alone writes the binary results file; when its writes fail
    (/dev/full: the header at swmm_start on the 30 x 30 grid, a reporting
    period's record on the 6 x 6 one, whose header fits stdio's buffer) every
    rank returns an error from the same call instead of going on into a
    collective rank 0 never reaches (api.cpp syncError)."""
    inp = _grid(tmp_path, n, n, route_step=5.0, variable_step=0.75, diameter=1.0, q=0.3)
    parts = _run_workers(inp, 100000, tmp_path, 2, "host", "werr", extra_env={"WORKER_OUT0": "/dev/full"},
                         timeout=300)
    codes = [tuple(int(c) for c in p["codes"]) for p in parts]
    assert codes[0] == codes[1] and any(codes[0]), codes
    assert {c for c in codes[0] if c} <= {307, 309}, codes


@pytest.mark.gpu
@pytest.mark.parametrize("case,transport", [("example_steady", "host"), ("example_steady_var", "host"),
                                            ("example_steady_pump", "host"), ("example_steady", "ipc"),
                                            ("example_steady_pump", "ipc")])
def test_steady_state_skipping_ranks_bitwise(case, transport, tmp_path):
    """SKIP_STEADY_STATE with two ranks (routing.c:236-244, 383-395): each
    step's inflow test (and pump switching, routing.c:224) and the previous
    step's system flow totals are reduced over the ranks, so every rank skips
    the same steps.  The owned state is bitwise the one-GPU run's and the
    binary results file rank 0 writes is byte-identical to the one-GPU file
    (the reference fixtures' networks: a hydrograph that settles; with pumps,
    storage units and pollutants)."""
    import shutil
    import _golden
    inp = str(tmp_path / (case + ".inp"))
    shutil.copy(_golden.inp(case), inp)
    one = _run_workers(inp, 100000, tmp_path, 1, "host", "one", save=True)[0]
    parts = _run_workers(inp, 100000, tmp_path, 2, transport, "two", save=True)
    if case == "example_steady_pump":
        # the regulators and pumps tie every node into one end-node group:
        # rank 0 owns the whole network and rank 1 nothing, so rank 1 (no
        # pumps, no inflows) skips exactly the steps rank 0's pump switches
        # and inflow changes veto only through the reduced change flag
        assert (parts[0]["node_owner"] == 0).all()
    else:
        assert all((p["node_owner"] == r).any() for r, p in enumerate(parts))
    _assert_bitwise(parts, one)
    assert open(str(tmp_path / "two_r0.out"), "rb").read() == open(str(tmp_path / "one_r0.out"), "rb").read()


@pytest.mark.gpu
def test_rccl_single_rank_bitwise(tmp_path):
    inp = _grid(tmp_path, 30, 30, route_step=5.0, variable_step=0.75, diameter=1.0, q=0.1)
    one = _run_workers(inp, 80, tmp_path, 1, "host", "plain")[0]
    rc = _run_workers(inp, 80, tmp_path, 1, "rccl", "rccl")[0]
    for k in one:
        if k.startswith(("node.", "link.")):
            np.testing.assert_array_equal(rc[k], one[k], err_msg=k)
    np.testing.assert_array_equal(rc["counters"], one["counters"])


@pytest.mark.gpu
def test_two_ranks_match_one_gpu_4m(tmp_path):
    """BASELINE configs[4] at full size: bench.py's 4m preset, a 1414 x 1414
    grid of 3,995,965 conduits, split into two row strips (host transport, both
    ranks on this box's GPU) against one GPU, in the benchmark's regime.  One
    GPU spins the network up for 2000 s and saves a hot start file; both runs
    restart from it for 15 steps, which surcharge and do not all converge;
    the two strips (host and IPC transports) and bench.py's default
    two-region partition (IPC) are bitwise equal to one GPU."""
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    cfg = bench.PRESETS["4m"]
    n = cfg["grid"]
    hs = str(tmp_path / "spin.hsf")
    kw = dict(route_step=cfg["route_step"], variable_step=cfg["variable_step"],
              diameter=cfg["diameter"], q=cfg["q"], report_all=False)
    spin = str(tmp_path / "spin.inp")
    netgen.write_grid(spin, n, n, end_time="00:33:20", files='SAVE HOTSTART "%s"' % hs, **kw)
    _run_workers(spin, 100000, tmp_path, 1, "host", "spin")
    assert os.path.getsize(hs) > 0
    inp = str(tmp_path / "g4m.inp")
    netgen.write_grid(inp, n, n, end_time="06:00:00", files='USE HOTSTART "%s"' % hs, **kw)
    steps = 15
    one = _run_workers(inp, steps, tmp_path, 1, "host", "one")[0]
    st, its, nonconv = one["counters"]
    assert one["link.newFlow"].size == 3995965
    assert nonconv > 0 and its / st > 3.0, one["counters"]
    assert (one["node.newDepth"][:-1] > cfg["diameter"]).sum() > 1000
    for transport in ("host", "ipc"):
        parts = _run_workers(inp, steps, tmp_path, 2, transport, "two_" + transport)
        assert all(_transport_of(p) == transport for p in parts)
        _assert_bitwise(parts, one)
    # bench.py's default partition with two ranks: two regions from the
    # calibration record (profiles/partition_weights.json), over IPC
    w, rec = bench.partition_weights(bench.workload_name("4m", cfg, n), n, n, n * n + 1)
    if w is not None:
        wpath = str(tmp_path / "w4m.npy")
        np.save(wpath, w)
        env = {"WORKER_WEIGHTS": "file:" + wpath, "WORKER_PARTMODE": "two_region"}
        parts = _run_workers(inp, steps, tmp_path, 2, "ipc", "two_region", extra_env=env)
        owner = parts[0]["node_owner"]
        assert (owner[n * (n - 20):n * n] == 0).any() and (owner[n * (n - 20):n * n] == 1).any()
        _assert_bitwise(parts, one)
