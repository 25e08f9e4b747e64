/*
 * swmm5_mi355x.h -- extension entry points of libswmm5_mi355x.so that have no
 * counterpart in the reference API.  They exist for measurement, testing and
 * the multi-GPU driver; a drop-in caller never needs them.
 */
#ifndef SWMM5_MI355X_EXT_H
#define SWMM5_MI355X_EXT_H

#include "swmm5.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Host-only start: builds the initial state exactly as swmm_start would
 * (project_init + routing init, reference swmm5.c:345-393) but never touches
 * the GPU.  Lets CPU-only tests compare parsing/validation/initialisation
 * against the reference.  swmm_step is an error after this call. */
int    DLLEXPORT swmmx_startHost(void);

/* Write the engine's full-precision state (static parameters + current
 * dynamic state, synchronised from HBM) as a SWDUMP1 record file, the format
 * of oracle/refdump.c.  Returns 0 or an error code. */
int    DLLEXPORT swmmx_exportState(const char *path);

/* Copy one named fp64 state array (e.g. "node.newDepth", "link.newFlow")
 * from the engine (device-synchronised) into dst[0..n).  Returns the number of
 * elements copied or -1 if the name is unknown. */
long   DLLEXPORT swmmx_getArray(const char *name, double *dst, long n);

/* Overwrite one named fp64 state array (host mirror and HBM). */
long   DLLEXPORT swmmx_setArray(const char *name, const double *src, long n);

/* Run n routing steps back to back (same as n calls of swmm_step). */
int    DLLEXPORT swmmx_runSteps(int n, double *elapsedTime);

/* Counters: [0] total routing steps, [1] total Picard iterations,
 * [2] non-converging steps, [3] Picard iterations of the last step,
 * [4] true conduits, [5] nodes, [6] conduits updated (not bypassed) by the
 * Picard iterations >= 1 timed since swmmx_setTiming(1), [7] conduits handled
 * by the streaming link kernel, [8] nodes that re-gathered their conduits in
 * the timed iterations >= 2 (the others kept their previous sums), [9] timed
 * iterations >= 2, [10] timed iterations >= 1, [11] [12] [13] [14] steps
 * launched with the unrolled, k_tail, k_sparse and list step graphs, [15] 1
 * when the outfall depths of iterations >= 2 are found in the next link
 * launch (deferred outfall prologue), [16] [17] [18] retired (the fused and
 * compact step graphs of rounds 4-5, removed; always 0).
 * Synchronises with the device. */
int    DLLEXPORT swmmx_getCounters(long long *out, int n);

/* Device kernel timing (steps run as eager launches while enabled; each timed
 * kernel is launched with hipExtLaunchKernelGGL, whose start/stop events carry
 * the kernel's own execution timestamps -- the durations rocprofv3's kernel
 * trace reports).  mode=1 enables, 0 disables; swmmx_getKernelTimes returns,
 * per kernel class, the number of timed launches and their total
 * milliseconds:  out[2*k] = launches, out[2*k+1] = ms;
 *   k: 0 link momentum, Picard iteration 0 (k_link<first>: every conduit),
 *      1 node update of iteration 0, 2 step end (k_step_end .. k_finalize),
 *      3 quality, 4 link momentum, executed iterations >= 1 (bypassed
 *      conduits skipped), 5 node update of iteration 1, 6 node updates of the
 *      executed iterations >= 2, 7 k_sparse + k_unfreeze, 8 ghost-link
 *      exchange of an iteration (several ranks: pack .. unpack on the routing
 *      stream), 9 convergence-flag exchange of an iteration (several ranks).
 * Returns the number of classes written. */
int    DLLEXPORT swmmx_setTiming(int mode);
int    DLLEXPORT swmmx_getKernelTimes(double *out, int n);

/* Host-side evaporation replay (after swmmx_startHost only: the project
 * cannot step afterwards): the evaporation rate (ft/s) climate_setState
 * gives routing steps starting at elapsedMsec[0..n-1] ms after the start, in
 * that order -- constant / monthly / time-series / climate-file / Hargreaves
 * rates with the monthly adjustments.  Returns n, or -(error code). */
long   DLLEXPORT swmmx_evapReplay(const double *elapsedMsec, long n, double *rates);

/* Algorithmic bytes per launch of each kernel class (the byte model of
 * DESIGN.md), same class order as above: the average over the launches timed
 * since swmmx_setTiming(1) (class 4 counts the conduits actually updated),
 * or the model value for a full launch when nothing has been timed. */
int    DLLEXPORT swmmx_getKernelBytes(double *out, int n);

/* Per Picard iteration k of the steps timed since swmmx_setTiming(1), seven
 * values each (out[7k .. 7k+6]): iterations run, conduits updated (not
 * bypassed), nodes that gathered their conduits, nodes updated (not frozen),
 * relaxation-only node updates, k_link ms, k_node ms.  Returns the number of
 * values available (7 x MAX_TRIALS once a step was timed). */
int    DLLEXPORT swmmx_getIterationStats(double *out, int n);

/* Average duration (microseconds) of `reps` back-to-back launches of one
 * kernel on the live state: which = 0 link momentum of Picard iteration 0,
 * 1 node update of iteration 0.  The launches are of separate instantiations
 * (k_link<..., probe = true>, k_node<..., probe = true>) so that a profiler's
 * per-kernel statistics keep them apart from the routing steps'.  Measurement
 * only: it advances the state, so call it after the run being measured
 * (every later swmm_step / swmm_stride returns error 500). */
int    DLLEXPORT swmmx_timeKernel(int which, int reps, double *avgUs);

/* The achievable HBM bandwidth: a STREAM triad
 * a[i] = b[i] + s c[i] over three arrays of nDoubles fp64 values (16-byte
 * lanes, arrays far beyond the MALL), `reps` launches timed with HIP events on
 * the current device.  out[0] triad GB/s (best launch), out[1] triad GB/s
 * (average), out[2] copy GB/s (best), out[3] bytes per triad launch.
 * Returns 0 or a negated HIP error. */
int    DLLEXPORT swmmx_streamTriad(long nDoubles, int reps, double *out);

/* Name of the compute backend ("hip:gfx950:<device name>" or "none"). */
int    DLLEXPORT swmmx_getBackend(char *buf, int size);

/* Select the HIP device ordinal used by swmm_start (default 0 / LOCAL_RANK). */
int    DLLEXPORT swmmx_setDevice(int ordinal);

/* ---- multi-GPU (one process per GPU) ----------------
 * The network is split by node blocks (a conduit follows its node1, an
 * outfall its conduit; pumps / regulators keep their end nodes on one rank).
 * A rank holds the nodes its links touch; the other ranks' links touching
 * them are its ghost links, whose {flow, surface areas, dq/dh} the owners send
 * every Picard iteration (RCCL ncclSend / ncclRecv between neighbours), so
 * every held node is summed over all its links in the reference's order and
 * the run is bitwise equal to one GPU.  Call before swmm_start, on every rank:
 *   rank 0: swmmx_ncclUniqueId(id, 128) and broadcast the id to the others;
 *   all:    swmmx_setPartition(rank, nranks, id, 128).
 * The binary results file and a saved hot start file are gathered from the
 * owning ranks and written by rank 0 (byte-identical to one GPU's); an error
 * one rank meets there is returned by every rank from the same call. */
int    DLLEXPORT swmmx_ncclUniqueId(void *out, int bytes);     /* returns bytes written */
int    DLLEXPORT swmmx_setPartition(int rank, int nranks, const void *ncclId, int idBytes);

/* Test transport: replace RCCL by a host callback that reduces n doubles in
 * place over the ranks (op 0 = sum, 1 = min) and returns 0 on success; steps
 * then run as eager launches.  fn = NULL restores RCCL. */
int    DLLEXPORT swmmx_setExchange(int (*fn)(double *buf, long n, int op, void *user), void *user);

/* Transport of the per-iteration exchange (after swmmx_setPartition and any
 * swmmx_setExchange, before swmm_start): 0 RCCL, 1 the host callback, 2 IPC --
 * each rank's kernels store the ghost links' values, the convergence flag and
 * the per-step reductions straight into the peers' memory (an uncached region
 * mapped with hipIpcOpenMemHandle), no collective library inside a step.  IPC
 * is bootstrapped over the host callback when one is set, else over RCCL; if
 * its start-up handshake fails on any rank every rank falls back to RCCL (with
 * a unique id) or the host callback.  Every wait behind an exchange is bounded
 * (SWMM5_XCHG_TIMEOUT seconds, default 60): a rank that stops answering makes
 * every rank's swmm_step return error 500 instead of hanging.  Returns 0, or
 * 500 for an unknown kind (or 1 without a callback). */
int    DLLEXPORT swmmx_setTransport(int kind);

/* The transport in use after swmm_start ("single", "rccl", "host", "ipc", or
 * a fallback note), written into buf. */
int    DLLEXPORT swmmx_getTransport(char *buf, int size);

/* Per-node work weights for the partition (global node order, n = the node
 * count; call after swmmx_setPartition, on every rank, before swmm_open's
 * partition is used): the contiguous node blocks then carry equal total
 * weight instead of equal node counts.  n = 0 restores equal counts. */
int    DLLEXPORT swmmx_setPartitionWeights(const double *w, int n);

/* Partition mode (with weights; call like swmmx_setPartitionWeights): 0 one
 * contiguous block of equal weight per rank (the default); 1 two regions --
 * the "hot" nodes (weight excess over the lightest node at least a quarter of
 * the largest excess: e.g. the surcharged band whose nodes run every sparse
 * Picard iteration) are cut into 2 nranks contiguous blocks of equal weight
 * dealt to ranks 0, 1, .., nranks-1, nranks-1, .., 0, the other nodes into
 * nranks blocks (rank r takes block r), so every rank gets an equal share of
 * the sparse work and of the full passes.  Returns 0 or 500 for an unknown
 * mode. */
int    DLLEXPORT swmmx_setPartitionMode(int mode);

/* Per node (global order, owned nodes of this rank; 0 elsewhere): its updates
 * in Picard iterations k >= 2 of the steps timed since swmmx_setTiming(1) --
 * the measured sparse work a weighted partition balances.  Returns the node
 * count or -1. */
int    DLLEXPORT swmmx_getNodeWork(double *out, int n);

/* Same layout: per node, the updates in iterations k >= 2 (list walks) of the
 * conduits whose node1 it is -- a conduit's owner follows its node1. */
int    DLLEXPORT swmmx_getConduitWork(double *out, int n);

/* Owning rank of every node (objType swmm_NODE) or link (swmm_LINK) under the
 * current partition; returns the object count. */
int    DLLEXPORT swmmx_getOwner(int objType, int *out, int n);

/* This rank's part of the current partition (after swmm_open), by name:
 * "lnode" held nodes (global indices), "llink" owned links, "lghost" ghost
 * links, "nbr" neighbour ranks, "sendOff" / "sendLink" links sent to each
 * neighbour (local owned indices), "recvOff" ghosts received from each,
 * "hasGhost" per held node, "rowptr" / "csr" the node -> link incidence the
 * node update sums (local link indices, ghosts after the owned links, bit 31
 * = the node is the link's node2).  Copies at most n values; returns the
 * array's length or -1. */
long   DLLEXPORT swmmx_getPartition(const char *name, int *out, long n);

/* Cross-section known-answer evaluation (test extension; needs no project).
 * Builds a section of reference shape code `type` from the four [XSECTIONS]
 * parameters p[4] (user units, length factor ucf, as xsect_setParams), then
 * fn = 0 writes its 11 parameters (yFull wMax ywMax aFull rFull sFull sMax
 * yBot aBot sBot rBot) to y; fn = 1..9 evaluates A(y), W(y), R(y), Y(A),
 * R(A), S(A), A(S), dS/dA, yCrit(q) at the n points x into y, on the host
 * (device = 0) or on the GPU with the kernels' code (device = 1).
 * Returns 0, 211 for invalid parameters, 500 when the device call fails. */
int    DLLEXPORT swmmx_xsect(int type, const double *p, double ucf, int fn,
                             const double *x, double *y, int n, int device);

#ifdef __cplusplus
}
#endif

#endif
