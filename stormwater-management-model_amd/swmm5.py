"""Python host mirror of the SWMM 5.2 engine API over libswmm5_mi355x.so.

A thin ctypes binding with the reference's entry-point names, argument meaning
and error convention (src/solver/include/swmm5.h:129-151; integer error codes
from src/solver/error.h, sticky once set).  It is what a pyswmm-style caller
would bind; the parity tests drive the engine through it exactly the way the
reference's own harnesses drive libswmm5.

The library is built in-tree (``make -C stormwater-management-model_amd/csrc``
or ``__graft_entry__.build()``); there is no pure-Python or CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SWMM5_LIB") or os.path.join(PKG_DIR, "libswmm5_mi355x.so")   # SWMM5_LIB: A/B builds

# swmm5.h enums (values are the reference's)
GAGE, SUBCATCH, NODE, LINK, SYSTEM = 0, 1, 2, 3, 100
JUNCTION, OUTFALL, STORAGE, DIVIDER = 0, 1, 2, 3
CONDUIT, PUMP, ORIFICE, WEIR, OUTLET = 0, 1, 2, 3, 4
NODE_TYPE, NODE_ELEV, NODE_MAXDEPTH, NODE_DEPTH, NODE_HEAD = 300, 301, 302, 303, 304
NODE_VOLUME, NODE_LATFLOW, NODE_INFLOW, NODE_OVERFLOW, NODE_RPTFLAG = 305, 306, 307, 308, 309
LINK_TYPE, LINK_NODE1, LINK_NODE2, LINK_LENGTH, LINK_SLOPE = 400, 401, 402, 403, 404
LINK_FULLDEPTH, LINK_FULLFLOW, LINK_SETTING, LINK_TIMEOPEN, LINK_TIMECLOSED = 405, 406, 407, 408, 409
LINK_FLOW, LINK_DEPTH, LINK_VELOCITY, LINK_TOPWIDTH, LINK_RPTFLAG = 410, 411, 412, 413, 414
STARTDATE, CURRENTDATE, ELAPSEDTIME, ROUTESTEP, MAXROUTESTEP = 0, 1, 2, 3, 4
REPORTSTEP, TOTALSTEPS, NOREPORT, FLOWUNITS = 5, 6, 7, 8

_lib = None


def kernel_source_sha() -> str:
    """sha256 (16 hex digits) over every engine source and header and the
    Makefile (compile flags): the stamp of the profiles/ records (in-graph
    kernel timing, PMC traffic) that bench.py reuses only for the same build
    inputs."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(PKG_DIR, "csrc")
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".h", ".cpp")) or f == "Makefile":
            h.update(f.encode())
            with open(os.path.join(d, f), "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


class EngineMissing(RuntimeError):
    pass


# kernel classes of swmmx_getKernelTimes / swmmx_getKernelBytes
KERNEL_CLASSES = ["link_momentum_first", "node_update_first", "step_end", "quality", "link_momentum_iter",
                  "node_update_iter1", "node_update_iter2plus", "sparse_tail", "ghost_exchange", "flag_exchange"]


def load_library(path: str | None = None):
    """Load the engine; raises EngineMissing (never falls back) if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise EngineMissing(
            "libswmm5_mi355x.so not built at %s -- run __graft_entry__.build()" % p)
    L = ctypes.CDLL(p)
    c_int, c_dbl, c_char_p = ctypes.c_int, ctypes.c_double, ctypes.c_char_p
    P = ctypes.POINTER
    sig = {
        "swmm_run": (c_int, [c_char_p, c_char_p, c_char_p]),
        "swmm_open": (c_int, [c_char_p, c_char_p, c_char_p]),
        "swmm_start": (c_int, [c_int]),
        "swmm_step": (c_int, [P(c_dbl)]),
        "swmm_stride": (c_int, [c_int, P(c_dbl)]),
        "swmm_end": (c_int, []),
        "swmm_report": (c_int, []),
        "swmm_close": (c_int, []),
        "swmm_getMassBalErr": (c_int, [P(ctypes.c_float)] * 3),
        "swmm_getVersion": (c_int, []),
        "swmm_getError": (c_int, [ctypes.c_char_p, c_int]),
        "swmm_getWarnings": (c_int, []),
        "swmm_getCount": (c_int, [c_int]),
        "swmm_getName": (None, [c_int, c_int, ctypes.c_char_p, c_int]),
        "swmm_getIndex": (c_int, [c_int, c_char_p]),
        "swmm_getValue": (c_dbl, [c_int, c_int]),
        "swmm_setValue": (None, [c_int, c_int, c_dbl]),
        "swmm_getSavedValue": (c_dbl, [c_int, c_int, c_int]),
        "swmm_writeLine": (None, [c_char_p]),
        "swmm_decodeDate": (None, [c_dbl] + [P(c_int)] * 7),
        "swmmx_startHost": (c_int, []),
        "swmmx_exportState": (c_int, [c_char_p]),
        "swmmx_getArray": (ctypes.c_long, [c_char_p, P(c_dbl), ctypes.c_long]),
        "swmmx_setArray": (ctypes.c_long, [c_char_p, P(c_dbl), ctypes.c_long]),
        "swmmx_runSteps": (c_int, [c_int, P(c_dbl)]),
        "swmmx_getCounters": (c_int, [P(ctypes.c_longlong), c_int]),
        "swmmx_setTiming": (c_int, [c_int]),
        "swmmx_getKernelTimes": (c_int, [P(c_dbl), c_int]),
        "swmmx_getKernelBytes": (c_int, [P(c_dbl), c_int]),
        "swmmx_getIterationStats": (c_int, [P(c_dbl), c_int]),
        "swmmx_getBackend": (c_int, [ctypes.c_char_p, c_int]),
        "swmmx_setDevice": (c_int, [c_int]),
        "swmmx_timeKernel": (c_int, [c_int, c_int, P(c_dbl)]),
        "swmmx_ncclUniqueId": (c_int, [ctypes.c_void_p, c_int]),
        "swmmx_setPartition": (c_int, [c_int, c_int, ctypes.c_void_p, c_int]),
        "swmmx_setExchange": (c_int, [ctypes.c_void_p, ctypes.c_void_p]),
        "swmmx_setTransport": (c_int, [c_int]),
        "swmmx_setPartitionWeights": (c_int, [P(c_dbl), c_int]),
        "swmmx_getNodeWork": (c_int, [P(c_dbl), c_int]),
        "swmmx_getConduitWork": (c_int, [P(c_dbl), c_int]),
        "swmmx_setPartitionMode": (c_int, [c_int]),
        "swmmx_getTransport": (c_int, [ctypes.c_char_p, c_int]),
        "swmmx_getOwner": (c_int, [c_int, P(c_int), c_int]),
        "swmmx_getPartition": (ctypes.c_long, [c_char_p, P(c_int), ctypes.c_long]),
        "swmmx_xsect": (c_int, [c_int, P(c_dbl), c_dbl, c_int, P(c_dbl), P(c_dbl), c_int, c_int]),
        "swmmx_evapReplay": (ctypes.c_long, [P(c_dbl), ctypes.c_long, P(c_dbl)]),
        "swmmx_streamTriad": (c_int, [ctypes.c_long, c_int, P(c_dbl)]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(L, name) and os.environ.get("SWMM5_LIB"):
            continue                    # an older build taken for an A/B comparison
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = L
    return L


def xsect(code: int, p, fn: int, x=None, device: bool = False):
    """Evaluate cross-section relation fn (0 = the 11 section parameters,
    1..9 = A(y) W(y) R(y) Y(A) R(A) S(A) A(S) dS/dA yCrit(q)) of a section of
    reference shape `code` with [XSECTIONS] parameters p (swmmx_xsect)."""
    import numpy as np
    L = load_library()
    pa = (ctypes.c_double * 4)(*[float(v) for v in p])
    xs = np.ascontiguousarray(np.zeros(11) if x is None else x, dtype=np.float64)
    ys = np.zeros(xs.size if fn else 11)
    P = ctypes.POINTER(ctypes.c_double)
    err = L.swmmx_xsect(code, pa, 1.0, fn, xs.ctypes.data_as(P), ys.ctypes.data_as(P), ys.size,
                        1 if device else 0)
    if err:
        raise ValueError("swmmx_xsect error %d" % err)
    return ys


def exported_symbols() -> list:
    """Names the C ABI must export (include/swmm5.h + include/swmm5_mi355x.h)."""
    names = []
    root = os.path.dirname(PKG_DIR)
    for h in ("swmm5.h", "swmm5_mi355x.h"):
        with open(os.path.join(root, "include", h)) as f:
            for line in f:
                line = line.strip()
                if "DLLEXPORT" in line and "(" in line and not line.startswith("#"):
                    head = line.split("(")[0].split()
                    names.append(head[-1].lstrip("*"))
    return names


class SWMM:
    """One engine instance (the engine is single-project per process, as the
    reference).  Methods return the reference's integer error codes."""

    def __init__(self, lib_path: str | None = None):
        self.L = load_library(lib_path)

    @staticmethod
    def _b(s):
        return s.encode() if isinstance(s, str) else s

    # --- lifecycle (swmm5.c:186-702)
    def run(self, inp, rpt, out):
        return self.L.swmm_run(self._b(inp), self._b(rpt), self._b(out))

    def open(self, inp, rpt, out):
        return self.L.swmm_open(self._b(inp), self._b(rpt), self._b(out))

    def start(self, save_results: bool = True):
        return self.L.swmm_start(1 if save_results else 0)

    def step(self):
        t = ctypes.c_double(0.0)
        err = self.L.swmm_step(ctypes.byref(t))
        return err, t.value

    def stride(self, seconds: int):
        t = ctypes.c_double(0.0)
        err = self.L.swmm_stride(int(seconds), ctypes.byref(t))
        return err, t.value

    def end(self):
        return self.L.swmm_end()

    def report(self):
        return self.L.swmm_report()

    def close(self):
        return self.L.swmm_close()

    # --- diagnostics
    def getMassBalErr(self):
        a, b, c = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        self.L.swmm_getMassBalErr(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return a.value, b.value, c.value

    def getVersion(self):
        return self.L.swmm_getVersion()

    def getError(self):
        buf = ctypes.create_string_buffer(512)
        code = self.L.swmm_getError(buf, 512)
        return code, buf.value.decode(errors="replace")

    def getWarnings(self):
        return self.L.swmm_getWarnings()

    def getCount(self, obj):
        return self.L.swmm_getCount(obj)

    def getName(self, obj, idx):
        buf = ctypes.create_string_buffer(256)
        self.L.swmm_getName(obj, idx, buf, 256)
        return buf.value.decode()

    def getIndex(self, obj, name):
        return self.L.swmm_getIndex(obj, self._b(name))

    def getValue(self, prop, idx=0):
        return self.L.swmm_getValue(prop, idx)

    def setValue(self, prop, idx, value):
        self.L.swmm_setValue(prop, idx, float(value))

    def getSavedValue(self, prop, idx, period):
        return self.L.swmm_getSavedValue(prop, idx, period)

    def writeLine(self, line):
        self.L.swmm_writeLine(self._b(line))

    def decodeDate(self, date):
        v = [ctypes.c_int() for _ in range(7)]
        self.L.swmm_decodeDate(float(date), *[ctypes.byref(x) for x in v])
        return tuple(x.value for x in v)

    # --- extensions (include/swmm5_mi355x.h)
    def start_host(self):
        return self.L.swmmx_startHost()

    def evap_replay(self, elapsed_msec) -> np.ndarray:
        """Evaporation rates (ft/s) of routing steps starting at these elapsed
        times, in order (swmmx_evapReplay; after start_host only)."""
        t = np.ascontiguousarray(elapsed_msec, dtype=np.float64)
        out = np.zeros(t.size)
        n = self.L.swmmx_evapReplay(t.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), t.size,
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        if n < 0:
            raise RuntimeError("swmmx_evapReplay error %d" % -n)
        return out

    def export_state(self, path):
        return self.L.swmmx_exportState(self._b(path))

    def get_array(self, name) -> np.ndarray:
        n = self.L.swmmx_getArray(self._b(name), None, 0)
        if n < 0:
            raise KeyError(name)
        a = np.empty(max(n, 1), dtype=np.float64)
        self.L.swmmx_getArray(self._b(name), a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), n)
        return a[:n]

    def set_array(self, name, values):
        a = np.ascontiguousarray(values, dtype=np.float64)
        return self.L.swmmx_setArray(self._b(name),
                                     a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), a.size)

    def run_steps(self, n):
        t = ctypes.c_double(0.0)
        err = self.L.swmmx_runSteps(int(n), ctypes.byref(t))
        return err, t.value

    def counters(self):
        a = (ctypes.c_longlong * 19)()
        self.L.swmmx_getCounters(a, 19)
        keys = ["steps", "iterations", "nonconverged", "last_iterations", "conduits", "nodes",
                "timed_updated", "streaming_conduits", "timed_gathered", "timed_gather_iters",
                "timed_iters1", "steps_unrolled", "steps_tail", "steps_sparse", "steps_list", "deferred_outfalls",
                "steps_fused", "steps_compact", "compact_grown"]
        return dict(zip(keys, list(a)))

    def set_timing(self, on: bool):
        return self.L.swmmx_setTiming(1 if on else 0)

    def kernel_times(self):
        a = (ctypes.c_double * (2 * len(KERNEL_CLASSES)))()
        n = self.L.swmmx_getKernelTimes(a, 2 * len(KERNEL_CLASSES))
        names = KERNEL_CLASSES
        return {names[k]: (a[2 * k], a[2 * k + 1]) for k in range(n)}

    def kernel_bytes(self):
        a = (ctypes.c_double * len(KERNEL_CLASSES))()
        n = self.L.swmmx_getKernelBytes(a, len(KERNEL_CLASSES))
        names = KERNEL_CLASSES
        return {names[k]: a[k] for k in range(n)}

    def iteration_stats(self):
        """Per Picard iteration of the timed steps (swmmx_getIterationStats):
        rows of (runs, conduits updated, nodes gathered, nodes updated,
        relaxation-only updates, k_link ms, k_node ms)."""
        import numpy as np
        n = self.L.swmmx_getIterationStats(None, 0)
        a = (ctypes.c_double * max(n, 1))()
        self.L.swmmx_getIterationStats(a, n)
        return np.array(a[:n]).reshape(-1, 7)

    def backend(self):
        buf = ctypes.create_string_buffer(256)
        self.L.swmmx_getBackend(buf, 256)
        return buf.value.decode()

    def time_kernel(self, which: int, reps: int = 20) -> float:
        v = ctypes.c_double(0.0)
        rc = self.L.swmmx_timeKernel(int(which), int(reps), ctypes.byref(v))
        if rc:
            raise RuntimeError("swmmx_timeKernel failed (%d)" % rc)
        return v.value

    def stream_triad(self, n_doubles: int = 64 << 20, reps: int = 20) -> dict:
        """The achievable HBM bandwidth: STREAM triad (and copy) GB/s on the
        current device, HIP-event timed (swmmx_streamTriad)."""
        out = (ctypes.c_double * 4)()
        rc = self.L.swmmx_streamTriad(int(n_doubles), int(reps), out)
        if rc:
            raise RuntimeError("swmmx_streamTriad failed (%d)" % rc)
        return {"triad_best_GBs": out[0], "triad_avg_GBs": out[1], "copy_best_GBs": out[2],
                "bytes_per_launch": out[3], "launches": int(reps)}

    def set_device(self, ordinal: int):
        return self.L.swmmx_setDevice(int(ordinal))

    # ---- multi-GPU (include/swmm5_mi355x.h) ----------------------------------
    def nccl_unique_id(self) -> bytes:
        buf = ctypes.create_string_buffer(128)
        n = self.L.swmmx_ncclUniqueId(buf, 128)
        if n <= 0:
            raise RuntimeError("ncclGetUniqueId failed (%d)" % n)
        return buf.raw[:n]

    def set_partition(self, rank: int, nranks: int, nccl_id: bytes | None = None):
        if nccl_id is None:
            return self.L.swmmx_setPartition(int(rank), int(nranks), None, 0)
        buf = ctypes.create_string_buffer(nccl_id, len(nccl_id))
        return self.L.swmmx_setPartition(int(rank), int(nranks), buf, len(nccl_id))

    def set_exchange(self, fn):
        """fn(array: numpy float64 view, op: 0 sum / 1 min) -> None, reducing in
        place over the ranks; None restores RCCL.  The ctypes trampoline is kept
        alive on this object."""
        if fn is None:
            self._xchg = None
            return self.L.swmmx_setExchange(None, None)
        import numpy as np
        CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_long,
                              ctypes.c_int, ctypes.c_void_p)

        def tramp(buf, n, op, user):
            try:
                fn(np.ctypeslib.as_array(buf, shape=(n,)), op)
                return 0
            except Exception:           # noqa: BLE001 -- reported as an engine error
                return 1
        self._xchg = CB(tramp)
        return self.L.swmmx_setExchange(ctypes.cast(self._xchg, ctypes.c_void_p), None)

    TRANSPORTS = {"rccl": 0, "host": 1, "ipc": 2}

    def set_transport(self, kind: str):
        """Transport of the per-iteration exchange (swmmx_setTransport): "rccl",
        "host" (the set_exchange callback) or "ipc" (device stores into the
        peers' memory; bootstrapped over the callback when one is set)."""
        return self.L.swmmx_setTransport(self.TRANSPORTS[kind])

    def set_partition_weights(self, w):
        """Per-node work weights of the partition (swmmx_setPartitionWeights);
        None or empty: equal node counts."""
        import numpy as np
        if w is None or len(w) == 0:
            return self.L.swmmx_setPartitionWeights(None, 0)
        a = np.ascontiguousarray(w, dtype=np.float64)
        self._pw = a
        return self.L.swmmx_setPartitionWeights(a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), a.size)

    def set_partition_mode(self, mode):
        """Partition mode (swmmx_setPartitionMode): "contiguous" (0) or "two_region" (1)."""
        m = {"contiguous": 0, "two_region": 1}.get(mode, mode)
        return self.L.swmmx_setPartitionMode(int(m))

    def node_work(self, conduits: bool = False):
        """Per-node updates in iterations k >= 2 of the timed steps (owned
        nodes); conduits: the updates of the conduits each node is node1 of."""
        import numpy as np
        n = self.getCount(NODE)
        a = np.zeros(max(n, 1))
        fn = self.L.swmmx_getConduitWork if conduits else self.L.swmmx_getNodeWork
        fn(a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), n)
        return a[:n]

    def transport(self) -> str:
        if not hasattr(self.L, "swmmx_getTransport"):     # an older build (SWMM5_LIB A/B runs)
            return "single"
        buf = ctypes.create_string_buffer(256)
        self.L.swmmx_getTransport(buf, 256)
        return buf.value.decode()

    def partition_array(self, name: str):
        """This rank's part of the partition (swmmx_getPartition)."""
        import numpy as np
        n = self.L.swmmx_getPartition(self._b(name), None, 0)
        if n < 0:
            raise KeyError(name)
        a = (ctypes.c_int * max(n, 1))()
        self.L.swmmx_getPartition(self._b(name), a, n)
        return np.array(a[:n], dtype=np.int64)

    def owners(self, obj_type: int):
        import numpy as np
        n = self.getCount(obj_type)
        a = (ctypes.c_int * max(n, 1))()
        self.L.swmmx_getOwner(obj_type, a, n)
        return np.array(a[:n], dtype=np.int32)
