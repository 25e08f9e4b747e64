// dw_kernels.hip -- gfx950 kernels and the HBM-resident router.
//
// One routing step (reference: routing_execute -> flowrout_execute ->
// dynwave_execute, src/solver/routing.c:203-265, dynwave.c:224-262) is:
//
//   for k in 0 .. MaxTrials-1:                      (graph nodes, early exit)
//     k_link<k==0>   one thread per conduit: Saint-Venant momentum update
//                    (dwflow_findConduitFlow, dwflow.c:57-293); iteration 0
//                    also rotates link state (link_setOldHydState, a2 <- a1)
//     k_node<k==0>   one thread per node: CSR gather of incident-link flows in
//                    link-index order (= the reference's serial scatter,
//                    dynwave.c:398-411, 528-589, so node sums are bit-exact),
//                    outfall depth (link.c:728-766) and continuity/depth update
//                    (setNodeDepth, dynwave.c:636-762); wave-level ballot of the
//                    convergence test (dynwave.c:618) into one flag per iteration
//   k_qual_node    pollutant advection (qualrout.c:100-142): node mixing, then
//                  each link updated by the thread of its upstream node
//   k_step_end     capacity-limited links, outfall system outflow, flow totals
//                  and Courant-step partials (dynwave.c:349-378, 799-921,
//                  routing.c:841-925)
//   k_finalize     one block: deterministic fixed-order reduction of the block
//                  partials, Picard-step count, next variable step.
//
// Everything is fp64 and compiled with -ffp-contract=off: apart from OCML vs
// glibc ulps in pow/exp/sqrt/sin/cos the arithmetic is the reference's.
// No MFMA: the path is HBM-bandwidth bound (DESIGN.md has the byte model).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstddef>
#include <map>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <unistd.h>

#include <rccl/rccl.h>

#include "router.h"
#include "xsect.h"
#include "culvert.h"
#include "storage.h"
#include "regulators.h"

namespace swx {

#define HIPCHECK(x)                                                                  \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fail(std::string(#x) + ": " + hipGetErrorString(e_));                    \
            return err_ ? err_ : 500;                                                \
        }                                                                            \
    } while (0)

// a bounded wait (waitDone) inside a Router method: its message becomes the router's error
#define WAITCHECK(x)                                                                 \
    do {                                                                             \
        if ((x) != 0) {                                                              \
            fail(d_->xerrMsg);                                                       \
            return err_ ? err_ : 500;                                                \
        }                                                                            \
    } while (0)

constexpr int kBlock = 256;
// phase probe slots per Picard iteration (Params::probe): link entry (min),
// link exit, link exit of workgroups with list work, node entry (min), last
// node workgroup's entry, block 0's outfall prologue end, node exit, node
// exit of block 0
enum { PR_L_IN = 0, PR_L_OUT, PR_L_WORK, PR_N_IN, PR_N_LAST_IN, PR_N_PRO, PR_N_OUT, PR_N_B0,
       PR_P_STAGED, PR_P_YN, PR_P_YC, PR_L_SCAN, PR_L_STAGED, kProbeSlots };
// per-block partials written by k_step_end: [0] outflow [1] flooding [2] extra
// external inflow [3] evap [4] seep (sums), [5] link Courant step [6] node
// Courant step (min, with their first-occurrence indices in [8] [9]),
// [7] system outfall flow (sum)
constexpr int kNumPartials = 11;
__host__ __device__ inline bool partialIsMin(int q) { return q == 5 || q == 6; }
constexpr int kTimeLevels = 6;     // TIMELEVELS (objects.h:941)
constexpr int kQualBatch = 4;      // pollutants whose node mass inflow k_qual_node sums in one link pass
constexpr int kQGather = 4;        // CSR entries k_qual_node loads together
constexpr int kDtRing = 4;          // host-mapped per-step dt ring (k_finalize -> host)
constexpr int kLinkWavesDefault = 3;   // measured best on MI355X
constexpr double kTailIters = 2.5;     // auto mode: k_tail while steps average at most this many iterations

// ---- packed per-link flags -------------------------------------------------
enum : uint32_t {
    LF_XTYPE = 0x1Fu,             // bits 0-4 cross-section type
    LF_BARREL_SHIFT = 5,          // bits 5-12 barrels
    LF_LOSSES = 1u << 13,
    LF_FLAP = 1u << 14,
    LF_N1_OUTFALL = 1u << 15,
    LF_N2_OUTFALL = 1u << 16,
    LF_N1_OFLAP = 1u << 17,       // node1 is an outfall with a flap gate
    LF_N2_OFLAP = 1u << 18,
    LF_SEEP = 1u << 19,           // seepage > 0 or evaporation active
    LF_QLIMIT = 1u << 20,
    LF_DIRNEG = 1u << 21,
    LF_COLD = 1u << 22,           // an invert offset: may need normal/critical depth
    LF_NC = 1u << 23,             // pump / orifice / weir / outlet (k_nc; also LF_COLD)
    LF_PUMP = 1u << 24,
    LF_DUMMY = 1u << 31,          // a DUMMY conduit (with LF_NC only: bit 31 is a geometry-id bit of streaming conduits)
    LF_CULVERT_SHIFT = 25,        // bits 25-30 culvert code (cold conduits only)
    LF_GEOM_SHIFT = 25,           // bits 25-31 geometry id (streaming conduits, kFast only)
};
// kFast: the streaming conduits' distinct circular sections (at most kGeomMax)
// are one table staged into LDS behind the circular tables; a conduit carries
// its section's id in LF_GEOM_SHIFT instead of loading 7 geometry doubles
constexpr int kGeomMax = 128;
constexpr int kGeomVals = 9;      // yFull wMax aFull rFull sFull sMax ywMax, 1/yFull (divdd.h pair)
constexpr int kCtFast = 5 * SWX_CIRC_N + kGeomVals * kGeomMax;
// ---- packed per-node flags -------------------------------------------------
enum : uint32_t {
    NF_TYPE = 0x3u,               // node type
    NF_OTYPE_SHIFT = 2,           // outfall type, 3 bits
    NF_DEGNEG = 1u << 5,          // degree < 0 (upstream terminal)
    NF_CANPOND = 1u << 6,
    NF_SHARED = 1u << 7,          // multi-GPU: touched by conduits of several ranks
    NF_REPLICA = 1u << 8,         // multi-GPU: replica of a node another rank owns
    NF_DEG0 = 1u << 9,            // degree 0 (no outflow link; massbal.c:622)
    NF_DEFER = 1u << 10,          // end node of a non-conduit link: updated by k_nc
};
// ---- packed link state word ------------------------------------------------
// bits 0-3 flowClass, 4-7 fullState code (0 / 8 / 9 / 10), 8 normalFlow,
// 9 capacityLimited, 10 inletControl
__host__ __device__ inline int stFlowClass(int s) { return s & 0xF; }
__host__ __device__ inline int stFullState(int s) { return (s >> 4) & 0xF; }

struct StepCtl {
    double dt;                    // step length used by the current step
    double dtNext;                // variable step computed at step end
    double variableStep;          // dynwave.c:84 VariableStep
    int lastSteps;
    int varStepOff;               // swmm_setValue(ROUTESTEP) mid-run: CourantFactor = 0
    long long totalSteps, totalIters, nonConverge;
    double stepTot[kNumPartials];     // this step's system totals (rates)
    double prevStepTot[kNumPartials]; // previous step's totals (massbal half step)
    double flowTot[kNumPartials];     // accumulated volumes
    double latTot[4];                 // {dwInflow, exInflow, exOutflow} rates of this step
    double newRoutingTime;            // msec (swmm5.c / routing.c clock mirror)
    double routingDuration;           // msec
    double routeStep;                 // fixed step (sec)
    double evapRate;                  // Evap.rate (ft/s) of this step (host: climate_setState)
    double hydconFactor;              // Adjust.hydconFactor (conduit seepage, storage exfiltration)
    double recoveryFactor;            // Evap.recoveryFactor (Green-Ampt moisture recovery)
    unsigned tailBar;             // k_tail's grid-barrier arrivals (zeroed by k_link<first>)
    int tailErr;                  // k_tail gave up waiting at a barrier (never expected)
    int qualPar;                  // quality buffer holding the latest concentrations (Params::nQual)
    // SKIP_STEADY_STATE (routing.c:383-395): steadyOk -- the previous step's
    // flow error was within SYS_FLOW_TOL (k_finalize); steadyChanged -- a
    // lateral or outfall inflow changed by more than LAT_FLOW_TOL (k_steady)
    int steadyOk, steadyChanged;
    // several ranks: [0..5] this step's system inflow / outflow rates for the
    // flow-error test, summed over the ranks between k_finalize's phases;
    // [6] > 0 when some rank's k_steady saw a changed inflow or a pump to
    // switch (summed over the ranks before the step's iterations)
    double steadyIO[8];
    double stepRed[kNumPartials];     // this step's reduced block partials (k_finalize)
    // run statistics (stats.c): report-period step count / span, max system
    // outfall flow, routing time-step statistics (stats_updateTimeStepStats)
    double statsStart;                // ReportStart (DateTime)
    double dateBase, dateSecs0;       // floor(StartDateTime), its time of day (sec)
    long long reportStepCount;
    double routingTimeSpan, maxOutfallFlow;
    double tsMin, tsMax, tsRoutingTime, tsSteadyTime;
    long long tsCount, tsTrials;
    long long tsCounts[kTimeLevels];
    double tsIntervals[kTimeLevels];
};

// ---- device-initiated multi-GPU exchange (XCHG_IPC) ----
// Every rank owns one uncached region (hipDeviceMallocUncached) that its peers
// map with hipIpcOpenMemHandle and write with 8-byte system-scope stores; the
// owner polls it.  Each 8-byte word is one granule {seq in the high 32 bits,
// 32 payload bits} written by ONE store, so a reader that sees the expected
// seq holds the payload without any fence (cdna guide, Guideline 16 R2); a
// double travels as two granules.  The sequence numbers live per rank in
// XCtl, advance identically on every rank (every rank runs the same
// exchanges: an iteration after convergence skips them everywhere), and pick
// one of two buffers by parity, so a fast rank can run one exchange ahead
// of a slow one without overwriting what the slow one has not read.
struct XCtl {
    unsigned ghostSeq;            // per-iteration ghost-link exchange (bumped by k_ipc_flag)
    unsigned qualSeq;             // per-step ghost concentrations (bumped by k_finalize)
    unsigned flagSeq;             // per-iteration convergence flag (k_ipc_flag)
    unsigned redSeq;              // small all-reduces (k_ipc_reduce: Courant limits, steady test)
};
struct XPeer {                    // a neighbour's receive areas, as mapped into this process
    unsigned long long *ghost, *qual;
    int nGhost, pad;
};
constexpr int kRedMax = 8;        // doubles per k_ipc_reduce
enum { XK_GHOST = 1, XK_QUAL, XK_FLAG, XK_RED, XK_HELLO };

// device run statistics (stats.c TNodeStats / TLinkStats / TOutfallStats and
// massbal.c NodeInflow / NodeOutflow), one SoA array per field
struct StatsDev {
    double *avgDepth, *maxDepth, *maxDepthDate, *volFlooded, *timeFlooded, *timeSurch;
    double *timeCourant, *totLat, *maxLat, *maxInflow, *maxInflowDate, *maxOverflow;
    double *maxOverflowDate, *maxPonded;
    int* nonConv;
    double *mbIn, *mbOut, *mbPendIn, *mbPendOut;      // node volume totals + pending rates
    double *oAvgFlow, *oMaxFlow, *oLoad;               // outfalls ([p][node] loads)
    int* oPeriods;
    double *lMaxFlow, *lMaxFlowDate, *lMaxVeloc, *lMaxDepth, *lTimeNormal, *lTimeSurch, *lTimeInlet;
    double *lTimeFullUp, *lTimeFullDn, *lTimeFullFlow, *lTimeCapLim, *lTimeClass, *lTimeCourant;
    int *lTurns, *lTurnSign;
    const double* qFull;
    // storage units (TStorageStats, stats.c:212-228), per node
    double *sAvgVol, *sMaxVol, *sMaxVolDate, *sMaxFlow, *sEvap, *sExfil;
};

struct RareLink {
    const double *cIn, *cOut, *cAvg, *qLimit;
    double *evapLoss, *seepLoss;
};
struct Params {
    int nN, nL, P, maxTrials;
    // options
    int surchargeMethod, inertDamping, normalFlowLtd, allowPonding, varStep;
    int forceMainEqn;             // FM_H_W or FM_D_W (FORCE_MAIN_EQUATION)
    double crownCutoff, minSurfArea, headTol, courantFactor, minRouteStep, routeStep;
    // link static
    const int2* lnodes;
    const uint32_t* lflags;
    const double *inv1, *inv2, *off1, *off2;
    const double *yFull, *wMax, *ywMax, *aFull, *rFull, *sFull, *sMax, *yBot, *aBot, *sBot, *rBot;
    const double *length, *modLength, *roughFactor, *beta, *qMax, *qLimit, *slope;
    const double *cIn, *cOut, *cAvg, *seepRate;
    // link dynamic
    double *lNewFlow, *lOldFlow, *lNewDepth, *lOldDepth, *lNewVolume, *lOldVolume;
    double *a1, *a2, *q1, *dqdh, *froude, *sa1, *sa2, *evapLoss, *seepLoss, *setting;
    int* lstate;
    // node static
    const uint32_t* nflags;
    const double *invert, *fullDepth, *surDepth, *pondedArea, *yCrown, *fullVolume, *fixedStage;
    const double *crownElev;
    const int* rowptr;
    const int* csr;               // link index | (1<<31 if node is the link's node2)
    const int* csrOther;          // per CSR entry: the link's other end node (-1: not held here)
    const int* outfallLink;       // per node: its single link (outfalls) or -1
    // node dynamic
    double *nNewDepth, *nOldDepth, *nNewVolume, *nOldVolume, *inflow, *outflow, *overflow;
    double *newLat, *oldLat, *oldNetInflow, *oldFlowInflow, *oldSurfArea, *dYdT;
    int* conv;
    // node sums of the last gather (surface area, sum dq/dh; inflow/outflow
    // live in inflow/outflow) and a per-node "an incident conduit was updated
    // in this iteration" flag: a node whose conduits were all bypassed keeps
    // the sums of its previous gather (identical operands, identical sums)
    double *nSurf, *nDqdh;
    unsigned char* dirty;         // bit 0: an incident conduit was updated; bit 1: yRaw valid
    // A clean junction whose last update was plain (not surcharged, ponded or
    // flooded, no volume) has an unchanged unrelaxed depth yRaw = yOld + dV /
    // surfArea, so its next update is just the relaxation 0.5 yLast + 0.5 yRaw
    double *yRaw, *yMaxNP;        // yMaxNP = fullDepth + surDepth (non-ponding yMax)
    // frozen junctions: a clean plain junction that has converged and whose
    // relaxation stays inside [0, min(yCrown, yMax)] keeps converging, and its
    // later updates are the bare relaxation y <- 0.5 y + 0.5 yRaw; it is not
    // visited again until an incident conduit is updated, and its depth is
    // advanced on demand (frozenDepth).  frz: 0 = live; f > 0: frozen, the
    // stored depth is that of iteration f - 1
    unsigned char* frz;
    int freeze;                   // freezing enabled (headTol > 0)
    // storage units (node.c:170-179), per node (stShape -1: not a storage unit)
    const int* stShape;
    const double *stA0, *stA1, *stA2, *stFEvap;
    const int *stCOff, *stCN;     // area curve slice of curveX / curveY
    const double *curveX, *curveY;
    double ucfL, ucfV;            // UCF(LENGTH), UCF(VOLUME)
    double* nLosses;              // per node: this step's loss rate (storage evaporation)
    double* nEvapVol;             // per node: this step's evaporated volume
    double* nExfilVol;            // per node: this step's exfiltrated volume
    const int* exIdx;             // per node: its seepage object in exData (-1: none)
    double* exData;               // [n][kExVals] storage seepage objects (storage.h)
    double* hrt;                  // per node: storage hydraulic residence time (sec)
    int* ulist;                   // [2][nN] unconverged nodes of the last two iterations
    // sparse Picard tail (k_sparse): vlist[k & 1] = the nodes not frozen after
    // iteration k (k_node(1), then k_sparse), vcount[k] their number; wlist
    // the frozen junctions an iteration's conduit updates woke, wmark[n] = 1
    // while n is on it (deduplication)
    int* vlist;
    int2* vlistRow;               // [2][nN] the live nodes' CSR row bounds (k_node(1), k_node_list)
    int* vcount;
    int* wlist;
    int* wmark;
    // k_node_list's claim stamps: a frozen junction woken at iteration k of
    // step s is claimed by the one thread that exchanges its stamp to
    // s (MaxTrials + 1) + k first
    unsigned* nstamp;
    int* wcount;                  // [maxTrials] wake-list length of iteration k (list graph)
    // non-conduit links (k_nc), in link order
    int nNC, nDef;
    const int* ncLinks;           // [nNC] link index
    const NcLink* ncL;            // [nNC] static parameters
    double* ncCoef;               // [nNC][4] cOrif, cWeir, hCrit, cSurcharge
    double* ncTarget;             // [nNC] target setting
    double* ncSurf;               // [nNC] orifice / weir equivalent surface area
    double* ncQ;                  // [nNC] this iteration's raw flow (pumps)
    int* ncBypass;                // [nNC] bypassed in this iteration
    const int* defNodes;          // [nDef] deferred nodes (ends of non-conduit links)
    double* nPrevDepth;           // outfalls: depth before this iteration's prologue
    const int *qrowptr, *qcsr;    // CSR over all links (quality mass inflow, link order)
    double *pUtil, *pAvg, *pVol, *pEnergy, *pOffLow, *pOffHigh, *pMin, *pMax;   // PumpStats, per link
    int *pStarts, *pPeriods;
    const double* latIn;          // lateral inflow for this step
    // quality [p][object], two buffers per object kind: during a step the
    // previous step's concentrations are read from [qualPar] and the new ones
    // written to [qualPar ^ 1]; k_finalize flips StepCtl::qualPar, so the
    // reference's old <- new rotation (node_setOldQualState etc.) is free
    double* nQual[2];
    double* lQual[2];
    const double* qualIn;         // mass loads for this step [p][node]
    const double* kDecay;
    // misc
    const double* gTables;        // global copy of the 5x51 circular tables, then
                                  // (kFast) nGeom x kGeomVals section geometries
    int nGeom;
    const double* gShapeTab;      // SWX_SHAPE_TAB: tabulated shapes' geometry
    const double* gXTab;          // transect / custom-shape table blocks (Network::xTab)
    const int* lTabOff;           // per link: its block in gXTab (-1: none); null without any
    const double* lengthRaw;      // Conduit.length as input (findLimitedLinks); = length unless irregular
    const double* ofTab;          // tidal curves / stage series of outfalls: (x, y) pairs
    const int* ofOff;             // per node: {offset of its pairs in ofTab, count} (-1: none)
    double startDateTime;         // StartDateTime (days)
    double* partials;             // [nBlocksEnd][kNumPartials]
    int nBlocksEnd;
    StatsDev st;
    int multi;                    // partitioned (multi-GPU) run
    int countWork;                // timing mode: count updated conduits per iteration
    unsigned* nodeWork;           // timing mode: per node, its updates in iterations k >= 2 (partition weights)
    unsigned* nodeLinkWork;       // timing mode: per node, updates in iterations k >= 2 of the conduits it is node1 of
    // multi-GPU exchange (partition.h): link arrays hold this rank's owned
    // links [0, nL) and its ghost links [nL, nLs) (other ranks' links touching
    // a held node).  Each iteration k_xpack packs the owned links other ranks
    // hold as ghosts (sendLink) into xsend, xF values each; the received
    // values (xrecv, ghost order) are unpacked into the ghost slots by
    // k_xunpack before k_node sums every held node over all its links
    int nLs;                      // owned + ghost links (stride of [p][link] quality arrays)
    int nSend, nGhost, xF;
    const int* sendLink;
    double *xsend, *xrecv;
    // per Picard iteration k < maxTrials (sized from MAX_TRIALS): unconv[k] =
    // "some node did not converge in iteration k"; ucount[k] = nodes (and
    // outfalls) k_node listed for the next iteration's link walk; work[4][k]
    // timing-mode counters: conduits updated, nodes gathered, nodes updated
    // (not frozen), relaxation-only node updates
    int* unconv;
    int* ucount;
    int2* ulistRow;               // [2][nN] each listed node's CSR row bounds (rowptr[u], rowptr[u + 1])
    unsigned long long* work;
    // phase probe (SWMM5_PROBE=1, timing mode only; null otherwise): per
    // iteration k, kProbeSlots wall-clock stamps (probeMark)
    unsigned long long* probe;    // [k][slot][probeBlocks]
    int probeBlocks;
    double* hostDt;               // host-mapped rings: per-step dt (Router::launchedDt), then
                                  // the Picard iterations each step ran (auto k_tail choice)
    int nCold, nOutLinks;
    // per k_node(1) workgroup: its nodes not frozen after iteration 1 (the
    // live count, summed by k_step_end into partial 10 for the host's graph
    // choice); buildVlist: k_node(1) also lists them (vlist), set in the
    // graphs whose iterations >= 2 are list-driven (GM_SPARSE, GM_LIST)
    int* blockLive;
    int blockLiveN, buildVlist;
    // iterations 2 <= k < MaxTrials - 1: outfall depths deferred from k_node(k)
    // to the next walk (k_walk, deferredOutfalls); host-checked (Router init)
    int deferPro;
    // measurement only (SWMM5_STEPEND_SKIP, PMC attribution of k_step_end's
    // bytes; results are wrong with any bit set): 1 link statistics, 2 link
    // flow-class times, 4 link maxima, 8 node volume totals, 16 node
    // statistics, 32 Courant limits, 64 capacity-limited state
    int endSkip;
    int qualUnfreeze;             // k_qual_node also does k_unfreeze's work (launchStep)
    // the link arrays only conduits with local losses, a flow limit or
    // seepage touch, behind one pointer: the streaming conduit update reads
    // them through it inside those branches, so their base addresses are not
    // held in scalar registers across its loop (kFast)
    const struct RareLink* rare;
    const int* coldLinks;         // LF_COLD conduits, ascending
    const int* outLinks;          // conduits with an outfall end, ascending
    int outInl0, outInl1, outInl2, outInl3;   // outLinks[0..3] (-1: none), read without a load
    const int* outNodes;          // per outLinks entry: its outfall node (node2 first, link.c:743-753)
    int outNd0, outNd1, outNd2, outNd3;       // outNodes[0..3], read without a load
    const double* ofQcs;          // [nOutLinks][26] their critical flows at the enumeration's
                                  // depths i yFull / 25 (static geometry: k_outfall_qcs at init)
    StepCtl* ctl;
    // SKIP_STEADY_STATE: a step in steady state routes no flow (routing.c:
    // 236-244; StepCtl::steadyOk / steadyChanged, stepIsSteady)
    int skipSteady;
    double sysFlowTol, latFlowTol;
    // ---- XCHG_IPC (the structs above): ghost links' values, the convergence
    // flag and the per-step reductions go straight into the peers' memory
    int ipc;                      // 1: this transport
    int xRank, xRanks;            // rank and rank count (xRanks <= 64: one wave)
    const XPeer* xpeer;           // [nbr] the neighbours' ghost / quality areas
    const int* sendNbr;           // per send entry: neighbour index k
    const int* sendGi;            // per send entry: ghost index at that neighbour
    const int* ghostFrom;         // per ghost: sending rank (error reports)
    unsigned long long* ghostRx;  // [2][2 xF][nGhost] granules received
    unsigned long long* qualRx;   // [2][2 P][nGhost]
    unsigned long long* flagRx;   // [2][xRanks]
    unsigned long long* redRx;    // [2][xRanks][2 kRedMax]
    unsigned long long* abortW;   // this rank's abort word (any rank sets it)
    unsigned long long* const* peerFlag;    // [xRanks] every rank's flagRx (own included)
    unsigned long long* const* peerRed;     // [xRanks] redRx
    unsigned long long* const* peerAbort;   // [xRanks] abort words
    XCtl* xctl;
    int* xerr;                    // host-mapped failure record {code, kind, rank, seq}
    const int* hostAbort;         // host-mapped: the host gave up waiting
    long long xTimeout;           // wall-clock ticks a wait may take
    long long stallStep;          // test hook (SWMM5_XCHG_STALL): from this step on this rank posts nothing
    // shared nodes that freeze (multi-GPU): the unpack of iteration k >= 2
    // marks a held end of a ghost link whose received values changed
    // (bitwise) as stale (dirty), exactly as the walk marks the ends of the
    // conduits it updates, and wakes it if frozen (xwlist / xwcount[k], the
    // list graph's third item source); with every change seen, a node touched
    // by ghost links may reuse its sums, relax on its cached depth and freeze
    // like any other junction.  0: such nodes never do (SWMM5_SHARED_FREEZE=0)
    int xwake;
    int* xwlist;                  // [nN] frozen held nodes a changed ghost value woke at iteration k
    int* xwcount;                 // [maxTrials]
};
// this step is skipped as steady (isInSteadyState, routing.c:383-395): read by
// the launches of Picard iterations 0 and 1 (the later ones see iteration 1's
// convergence flag, which a skipped step leaves at 0)
__device__ __forceinline__ bool stepIsSteady(const Params& p)
{
    return p.skipSteady && p.ctl->steadyOk && !p.ctl->steadyChanged && !(p.ctl->steadyIO[6] > 0.0);
}

// ===========================================================================
//  device helpers
// ===========================================================================
// kFast: every streaming conduit is CIRCULAR and the surcharge method is not
// SLOT (host-checked); the shape switches and the slot branch then fold away.
// every section operand of link j loaded at once, whatever its shape (the
// outfall prologue: no load waits for the flag word)
__device__ __forceinline__ Geom loadGeomEager(const Params& p, int j, uint32_t f)
{
    Geom g;
    const double yb = p.yBot[j], ab = p.aBot[j], sb = p.sBot[j], rb = p.rBot[j];
    g.yFull = p.yFull[j];
    g.wMax = p.wMax[j];
    g.aFull = p.aFull[j];
    g.rFull = p.rFull[j];
    g.sFull = p.sFull[j];
    g.sMax = p.sMax[j];
    g.ywMax = p.ywMax[j];
    const int tabOff = p.lTabOff ? p.lTabOff[j] : -1;
    g.type = (int)(f & LF_XTYPE);
    const bool circ = g.type == G_CIRCULAR;
    g.yBot = circ ? 0.0 : yb;
    g.aBot = circ ? 0.0 : ab;
    g.sBot = circ ? 0.0 : sb;
    g.rBot = circ ? 0.0 : rb;
    if (!isBasicShape(g.type)) {
        int off = shapeTabOffset(g.type);
        if (off >= 0) g.tb = p.gShapeTab + off;
        else g.tb = (tabOff >= 0) ? p.gXTab + tabOff : nullptr;
    }
    return g;
}

template <bool kFast = false>
__device__ __forceinline__ Geom loadGeom(const Params& p, int j, uint32_t f, const double* ct = nullptr)
{
    Geom g;
    if (kFast) {                  // LDS geometry table (stageTables with kFast)
        const double* t = ct + 5 * SWX_CIRC_N + kGeomVals * (int)(f >> LF_GEOM_SHIFT);
        g.type = G_CIRCULAR;
        g.yFull = t[0]; g.wMax = t[1]; g.aFull = t[2]; g.rFull = t[3];
        g.sFull = t[4]; g.sMax = t[5]; g.ywMax = t[6];
        g.rYh = t[7]; g.rYl = t[8];
        g.yBot = g.aBot = g.sBot = g.rBot = 0.0;
        return g;
    }
    g.type = (int)(f & LF_XTYPE);
    g.yFull = p.yFull[j];
    g.wMax = p.wMax[j];
    g.aFull = p.aFull[j];
    g.rFull = p.rFull[j];
    g.sFull = p.sFull[j];
    g.sMax = p.sMax[j];
    g.ywMax = p.ywMax[j];
    if (g.type != G_CIRCULAR) {
        g.yBot = p.yBot[j];
        g.aBot = p.aBot[j];
        g.sBot = p.sBot[j];
        g.rBot = p.rBot[j];
    } else {
        g.yBot = g.aBot = g.sBot = g.rBot = 0.0;
    }
    if (!kFast && !isBasicShape(g.type)) {
        int off = shapeTabOffset(g.type);
        if (off >= 0) g.tb = p.gShapeTab + off;
        else g.tb = (p.lTabOff && p.lTabOff[j] >= 0) ? p.gXTab + p.lTabOff[j] : nullptr;
    }
    return g;
}

// dwflow.c:575-588
template <bool kFast = false>
__device__ __forceinline__ double slotWidth(const Params& p, const Geom& x, double y)
{
    if (kFast) return 0.0;
    double yNorm = y / x.yFull;
    if (p.surchargeMethod != SUR_SLOT || isOpen(x.type) || yNorm < p.crownCutoff) return 0.0;
    if (yNorm > 1.78) return 0.01 * x.wMax;
    return x.wMax * 0.5423 * exp(-pow(yNorm, 2.4));
}
// dwflow.c:592-605
// kAll: every shape (cold conduits); streaming conduits are basic shapes
template <bool kFast = false, bool kAll = false>
__device__ __forceinline__ double widthAt(const Params& p, const Geom& x, double y, const double* ct)
{
    double wSlot = slotWidth<kFast>(p, x, y);
    if (wSlot > 0.0) return wSlot;
    if (normDepth(x, y) >= p.crownCutoff && !isOpen(x.type)) y = p.crownCutoff * x.yFull;
    return getWofY<kAll>(x, y, ct);
}
// dwflow.c:609-619, 623-633
template <bool kAll = false>
__device__ __forceinline__ double areaAt(const Geom& x, double y, double wSlot, const double* ct)
{
    if (y >= x.yFull) return x.aFull + (y - x.yFull) * wSlot;
    return getAofY<kAll>(x, y, ct);
}
template <bool kAll = false>
__device__ __forceinline__ double hydRadAt(const Geom& x, double y, const double* ct)
{
    if (y >= x.yFull) return x.rFull;
    return getRofY<kAll>(x, y, ct);
}
// The same relations for a circular section (the kFast instantiation: no
// slot) given the depth's normalised value yn = normDepth(x, y) and its
// circular-table index part c = circIdx(yn): the operations of widthAt /
// areaAt / hydRadAt / linkFroude with the index part computed once per depth
__device__ __forceinline__ double circWidthAt(const Params& p, const Geom& x, double yn, const CircIdx& c,
                                              const double* ct)
{
    if (yn >= p.crownCutoff)                       // closed section: the width at the crown cutoff
        return x.wMax * lookup(normDepth(x, p.crownCutoff * x.yFull), SWX_TW(ct), SWX_CIRC_N);
    return x.wMax * circLookup(c, SWX_TW(ct));
}
__device__ __forceinline__ double circAreaAt(const Geom& x, double y, const CircIdx& c, const double* ct)
{
    if (y >= x.yFull) return x.aFull + (y - x.yFull) * 0.0;      // (no slot: wSlot = 0)
    if (y <= 0.0) return 0.0;
    return x.aFull * circLookup(c, SWX_TA(ct));
}
__device__ __forceinline__ double circHydRadAt(const Geom& x, double y, const CircIdx& c, const double* ct)
{
    if (y >= x.yFull) return x.rFull;
    return x.rFull * circLookup(c, SWX_TR(ct));
}
// link_getFroude (link.c:847-871) at depth y whose area a = A(y) (y < yFull:
// the caller's areaAt value) and width w = widthAt(y) were found already: the
// unclamped top width is w below the crown cutoff, else read again
__device__ __forceinline__ double circFroude(const Params& p, const Geom& x, double v, double y, double yn,
                                             const CircIdx& c, double a, double w, const double* ct)
{
    if (y <= 0.0001) return 0.0;
    if (x.yFull - y <= 0.0001) return 0.0;         // closed section
    const double wy = (yn >= p.crownCutoff) ? x.wMax * circLookup(c, SWX_TW(ct)) : w;
    const double hy = a / wy;
    return fabs(v) / sqrt(32.2 * hy);
}

// link.c:1334-1399 (DW branch); returns total loss rate, sets evap/seep
template <bool kAll>
__device__ double conduitLossRate(const Params& p, int j, const Geom& x, double tstep,
                                  double* evapOut, double* seepOut, const double* ct)
{
    double depth = 0.5 * (p.lOldDepth[j] + p.lNewDepth[j]);
    double evapLossRate = 0.0, seepLossRate = 0.0, totalLossRate = 0.0;
    if (depth > 0.0001) {
        double len = p.length[j];
        const double evapRate = p.ctl->evapRate;
        if (isOpen(x.type) && evapRate > 0.0) {
            double topWidth = getWofY<kAll>(x, depth, ct);
            evapLossRate = topWidth * len * evapRate;
        }
        double sr = p.seepRate[j];
        if (sr > 0.0) {
            double width;
            if (x.type == G_RECT_CLOSED) width = x.wMax;
            else {
                if (depth >= x.ywMax) depth = x.ywMax;
                width = getWofY<kAll>(x, depth, ct);
            }
            seepLossRate = sr * width * len;
            seepLossRate *= p.ctl->hydconFactor;
        }
        totalLossRate = evapLossRate + seepLossRate;
        double q = p.lNewVolume[j] / tstep;
        if (totalLossRate > q) {
            evapLossRate = evapLossRate * q / totalLossRate;
            seepLossRate = seepLossRate * q / totalLossRate;
            totalLossRate = q;
        }
    }
    *evapOut = evapLossRate;
    *seepOut = seepLossRate;
    return totalLossRate;
}

// depth of node i at Picard iteration m: a frozen junction (Params::frz)
// advances by the relaxation of setNodeDepth's plain branch (dynwave.c:
// 700-715, omega = 0.5, yNew = yOld + dV / surfArea = yRaw unchanged), the
// same operations the live update would have made
__device__ __forceinline__ double frozenDepthV(double y, double yr, int fz, int m)
{
    if (fz)
        for (int j = fz - 1; j < m; j++) y = (1.0 - 0.5) * y + 0.5 * yr;
    return y;
}
__device__ __forceinline__ double frozenDepth(const Params& p, int i, int fz, int m)
{
    return frozenDepthV(p.nNewDepth[i], fz ? p.yRaw[i] : 0.0, fz, m);
}

// dwflow.c:297-413.  kCold = false is the specialisation for links with both
// offsets zero (LF_COLD clear): z1 = z2 = 0 (at an outfall end too, since
// max(0, 0 - depth) = 0), so the branches that need normal / critical depth
// (root finders) are unreachable and are not compiled into the streaming
// kernel.
template <bool kCold>
__device__ __forceinline__ int flowClassOf(const Params& p, int j, const Geom& x, uint32_t f,
                                           double yn1, double yn2, double q, double h1, double h2,
                                           double y1, double y2, double* yC, double* yN,
                                           double* fasnh, const double* ct)
{
    double z1 = 0.0, z2 = 0.0;
    if (kCold) {
        z1 = p.off1[j];
        z2 = p.off2[j];
        if (f & LF_N1_OUTFALL) z1 = gmax(0.0, (z1 - yn1));
        if (f & LF_N2_OUTFALL) z2 = gmax(0.0, (z2 - yn2));
    }
    int fc = F_SUBCRIT;
    *fasnh = 1.0;
    if (y1 > 0.0001 && y2 > 0.0001) {
        if (q < 0.0) {
            if (kCold && z1 > 0.0) {
                *yN = linkYnorm(x, fabs(q), p.qMax[j], p.beta[j], ct);
                *yC = getYcrit(x, fabs(q), ct);
                double ycMin = gmin(*yN, *yC);
                if (y1 < ycMin) fc = F_UP_CRIT;
            }
        } else {
            if (kCold && z2 > 0.0) {
                *yN = linkYnorm(x, fabs(q), p.qMax[j], p.beta[j], ct);
                *yC = getYcrit(x, fabs(q), ct);
                double ycMin = gmin(*yN, *yC);
                double ycMax = gmax(*yN, *yC);
                if (y2 < ycMin) fc = F_DN_CRIT;
                else if (y2 < ycMax) {
                    if (ycMax - ycMin < 0.0001) *fasnh = 0.0;
                    else *fasnh = (ycMax - y2) / (ycMax - ycMin);
                }
            }
        }
    } else if (y1 <= 0.0001 && y2 <= 0.0001) {
        fc = F_DRY;
    } else if (y2 > 0.0001) {
        if (h2 < p.inv1[j] + (kCold ? p.off1[j] : 0.0)) fc = F_UP_DRY;
        else if (kCold && z1 > 0.0) {
            *yN = linkYnorm(x, fabs(q), p.qMax[j], p.beta[j], ct);
            *yC = getYcrit(x, fabs(q), ct);
            fc = F_UP_CRIT;
        }
    } else {
        if (h1 < p.inv2[j] + (kCold ? p.off2[j] : 0.0)) fc = F_DN_DRY;
        else if (kCold && z2 > 0.0) {
            *yN = linkYnorm(x, fabs(q), p.qMax[j], p.beta[j], ct);
            *yC = getYcrit(x, fabs(q), ct);
            fc = F_DN_CRIT;
        }
    }
    return fc;
}


// dwflow.c:57-293 -- one conduit, one Picard iteration
template <bool kFirst, bool kCold, bool kFast = false>
__device__ __forceinline__ void conduitFlow(const Params& p, int j, uint32_t f, int2 nn, int steps,
                                            double dt, const double* ct, double yn1, double yn2)
{
    const double omega = 0.5;
    (void)nn;                     // end-node depths arrive as yn1 / yn2
    const double off1 = kCold ? p.off1[j] : 0.0;     // hot links: both offsets are 0
    const double off2 = kCold ? p.off2[j] : 0.0;
    Geom x = loadGeom<kFast>(p, j, f, ct);
    double barrels = (double)((f >> LF_BARREL_SHIFT) & 0xFF);

    // iteration 0: link_setOldHydState (link.c:564-583), a2 <- a1 (dynwave.c:292)
    double oldFlow, oldDepth;
    if (kFirst) {
        double newFlowPrev = p.lNewFlow[j];
        oldFlow = newFlowPrev;
        oldDepth = p.lNewDepth[j];
        p.lOldFlow[j] = oldFlow;
        p.lOldDepth[j] = oldDepth;
        p.lOldVolume[j] = p.lNewVolume[j];
        double a1v = p.a1[j];
        p.a2[j] = a1v;
    } else {
        oldFlow = p.lOldFlow[j];
    }
    bool isClosed = (p.setting[j] == 0);
    double qOld = (barrels == 1.0) ? oldFlow : oldFlow / barrels;   // x / 1 == x
    double qLast = p.q1[j];
    double evapRate = 0.0, seepRate = 0.0;

    double inv1 = p.inv1[j], inv2 = p.inv2[j];
    double z1 = inv1 + off1;
    double z2 = inv2 + off2;
    double h1 = yn1 + inv1;
    double h2 = yn2 + inv2;
    h1 = gmax(h1, z1);
    h2 = gmax(h2, z2);
    double y1 = h1 - z1;
    double y2 = h2 - z2;
    y1 = gmax(y1, 0.0001);
    y2 = gmax(y2, 0.0001);
    if (kFast || p.surchargeMethod != SUR_SLOT) {
        y1 = gmin(y1, x.yFull);
        y2 = gmin(y2, x.yFull);
    }
    double aOld = kFirst ? p.a1[j] : p.a2[j];
    aOld = gmax(aOld, 0.0001);
    double length = p.modLength[j];

    // ---- findSurfArea (dwflow.c:417-550) ----
    int fc;
    double sa1 = 0.0, sa2 = 0.0;
    [[maybe_unused]] double nd1 = 0.0, nd2 = 0.0, ndM = 0.0, dMidF = 0.0, w1F = 0.0, wMidF = 0.0;
    [[maybe_unused]] CircIdx c1{}, c2{}, cM{};
    {
        double d1 = y1, d2 = y2, dMid, w1 = 0.0, w2, wMid = 0.0, fasnh = 1.0;
        double yNorm = (d1 + d2) / 2.0;
        double yCrit = yNorm;
        if (d1 >= x.yFull && d2 >= x.yFull) fc = F_SUBCRIT;
        else fc = flowClassOf<kCold>(p, j, x, f, yn1, yn2, qLast, h1, h2, y1, y2, &yCrit, &yNorm, &fasnh, ct);
        // Every wet class evaluates the top width at (d1, d2, dMid) after
        // adjusting one end; the widths are computed once, outside the switch,
        // so the geometry code is instantiated three times instead of fifteen.
        // (Widths a class does not use are pure and discarded.)
        switch (fc) {
        case F_UP_CRIT:
            d1 = yCrit;
            if (yNorm < yCrit) d1 = yNorm;
            d1 = gmax(d1, 0.0001);
            h1 = inv1 + off1 + d1;
            break;
        case F_DN_CRIT:
            d2 = yCrit;
            if (yNorm < yCrit) d2 = yNorm;
            d2 = gmax(d2, 0.0001);
            h2 = inv2 + off2 + d2;
            break;
        case F_UP_DRY: d1 = 0.0001; break;
        case F_DN_DRY: d2 = 0.0001; break;
        default: break;
        }
        if constexpr (kFast) {
            // the all-circular instantiation: the circular tables' index
            // parts at d1, d2 and their mean, shared by every table read at
            // those depths below (widths, areas, radii, Froude numbers)
            dMid = 0.5 * (d1 + d2);
            if (dMid < 0.0001) dMid = 0.0001;
            nd1 = normDepth(x, d1);
            nd2 = normDepth(x, d2);
            ndM = normDepth(x, dMid);
            c1 = circIdx(nd1);
            c2 = circIdx(nd2);
            cM = circIdx(ndM);
        }
        if (fc == F_DRY) {
            sa1 = 0.0001 * length / 2.0;
            sa2 = sa1;
        } else {
            if constexpr (kFast) {
                w1 = circWidthAt(p, x, nd1, c1, ct);
                w2 = circWidthAt(p, x, nd2, c2, ct);
                wMid = circWidthAt(p, x, ndM, cM, ct);
            } else {
                dMid = 0.5 * (d1 + d2);
                if (dMid < 0.0001) dMid = 0.0001;
                w1 = widthAt<kFast, kCold>(p, x, d1, ct);
                w2 = widthAt<kFast, kCold>(p, x, d2, ct);
                wMid = widthAt<kFast, kCold>(p, x, dMid, ct);
            }
            switch (fc) {
            case F_SUBCRIT:                                  // dwflow.c:460-472
                sa1 = (w1 + wMid) * length / 4.;
                sa2 = (wMid + w2) * length / 4. * fasnh;
                break;
            case F_UP_CRIT:                                  // dwflow.c:474-488
                sa2 = (wMid + w2) * length * 0.5;
                break;
            case F_DN_CRIT:                                  // dwflow.c:490-504
                sa1 = (w1 + wMid) * length * 0.5;
                break;
            case F_UP_DRY:                                   // dwflow.c:506-519
                sa2 = (wMid + w2) * length / 4.;
                if (off1 <= 0.0) sa1 = (w1 + wMid) * length / 4.;
                break;
            default:                                         // F_DN_DRY dwflow.c:521-534
                sa1 = (wMid + w1) * length / 4.;
                if (off2 <= 0.0) sa2 = (w2 + wMid) * length / 4.;
                break;
            }
        }
        y1 = d1;
        y2 = d2;
        if constexpr (kFast) {
            dMidF = dMid;
            w1F = w1;
            wMidF = wMid;
        }
    }
    p.sa1[j] = sa1;
    p.sa2[j] = sa2;

    double a1, r1, a2, aMid, rMid;
    double yMid = 0.5 * (y1 + y2);
    if constexpr (kFast) {
        // (yMid is dMid: both ends are at least 0.0001, so the floor never
        // applies; checked, with the index part recomputed otherwise)
        if (yMid != dMidF) {
            ndM = normDepth(x, yMid);
            cM = circIdx(ndM);
            wMidF = circWidthAt(p, x, ndM, cM, ct);
        }
        a1 = circAreaAt(x, y1, c1, ct);
        r1 = circHydRadAt(x, y1, c1, ct);
        a2 = circAreaAt(x, y2, c2, ct);
        aMid = circAreaAt(x, yMid, cM, ct);
        rMid = circHydRadAt(x, yMid, cM, ct);
    } else {
        double wSlot = slotWidth<kFast>(p, x, y1);
        a1 = areaAt<kCold>(x, y1, wSlot, ct);
        r1 = hydRadAt<kCold>(x, y1, ct);
        wSlot = slotWidth<kFast>(p, x, y2);
        a2 = areaAt<kCold>(x, y2, wSlot, ct);
        wSlot = slotWidth<kFast>(p, x, yMid);
        aMid = areaAt<kCold>(x, yMid, wSlot, ct);
        rMid = hydRadAt<kCold>(x, yMid, ct);
    }
    bool isFull = (y1 >= x.yFull && y2 >= x.yFull);
    double len0 = p.length[j];

    if (fc == F_DRY || fc == F_UP_DRY || fc == F_DN_DRY || isClosed || aMid <= 0.0001) {
        double a1n = 0.5 * (a1 + a2);
        p.a1[j] = a1n;
        p.q1[j] = 0.0;
        p.dqdh[j] = 32.2 * dt * aMid / length * barrels;
        p.froude[j] = 0.0;
        p.lNewDepth[j] = gmin(yMid, x.yFull);
        p.lNewVolume[j] = a1n * len0 * barrels;
        p.lNewFlow[j] = 0.0;
        if (f & LF_SEEP) {            // always 0 without LF_SEEP: not rewritten
            if constexpr (kFast) {
                p.rare->evapLoss[j] = 0.0;
                p.rare->seepLoss[j] = 0.0;
            } else {
                p.evapLoss[j] = 0.0;
                p.seepLoss[j] = 0.0;
            }
        }
        int old = p.lstate[j];
        p.lstate[j] = (old & ~0xF) | fc;   // fullState / normalFlow / inletControl untouched (dwflow.c:165-180)
        return;
    }

    double v = qLast / aMid;
    if (fabs(v) > 50.) v = 50. * gsgn(qLast);
    double froude;
    if constexpr (kFast) froude = circFroude(p, x, v, yMid, ndM, cM, aMid, wMidF, ct);
    else froude = linkFroude<kCold>(x, v, yMid, ct);
    p.froude[j] = froude;
    if (fc == F_SUBCRIT && froude > 1.0) fc = F_SUPCRIT;

    double sigma;
    if (froude <= 0.5) sigma = 1.0;
    else if (froude >= 1.0) sigma = 0.0;
    else sigma = 2.0 * (1.0 - froude);

    double rho = 1.0;
    if (!isFull && qLast > 0.0 && h1 >= h2) rho = sigma;
    double aWtd = a1 + (aMid - a1) * rho;
    double rWtd = r1 + (rMid - r1) * rho;

    if (p.inertDamping == DAMP_NO) sigma = 1.0;
    else if (p.inertDamping == DAMP_FULL) sigma = 0.0;
    if (isFull && !isOpen(x.type)) sigma = 0.0;

    double dq1;
    if (kCold && x.type == G_FORCE_MAIN && isFull)              // dwflow.c:212-214
        dq1 = dt * fmFricSlope(p.forceMainEqn, x, fabs(v), rMid);
    // the all-circular streaming instantiation (kFast: the benchmark grids)
    // takes the short form of pow (swxPowFriction, a few ulp); every other
    // network keeps OCML's pow: the ill-conditioned fixtures (mixed shapes,
    // culverts, offsets) amplify a last-bit difference into a chaotic value
    // -- with the short form example_shapes' final stored volume moved 1.1 %,
    // where all three reference builds agree
    else dq1 = dt * p.roughFactor[j] / (kFast ? swxPowFriction(rWtd) : pow(rWtd, 1.33333)) *
               fabs(v);
    // the three quotients by the conduit's length and the two by the
    // momentum denominator share a reciprocal pair each (divdd.h
    // recipDDFast: RN(a / b) exactly, with one division per divisor)
    double rLh, rLl;
    recipDDFast(length, &rLh, &rLl);
    double dq2 = divDD(dt * 32.2 * aWtd * (h2 - h1), length, rLh, rLl);
    double dq3 = 0.0, dq4 = 0.0;
    if (sigma > 0.0) {
        dq3 = 2.0 * v * (aMid - aOld) * sigma;
        dq4 = divDD(dt * v * v * (a2 - a1), length, rLh, rLl) * sigma;
    }
    double dq5 = 0.0;
    if (f & LF_LOSSES) {                                        // dwflow.c:554-571
        double losses = 0.0, qa = fabs(qLast);
        const double *cIn = p.cIn, *cOut = p.cOut, *cAvg = p.cAvg;
        if constexpr (kFast) {
            cIn = p.rare->cIn;
            cOut = p.rare->cOut;
            cAvg = p.rare->cAvg;
        }
        if (a1 > 0.0001) losses += cIn[j] * (qa / a1);
        if (a2 > 0.0001) losses += cOut[j] * (qa / a2);
        if (aMid > 0.0001) losses += cAvg[j] * (qa / aMid);
        dq5 = losses / 2.0 / length * dt;
    }
    double dq6 = 0.0;
    if (f & LF_SEEP) {
        if (!kFirst) oldDepth = p.lOldDepth[j];
        (void)oldDepth;
        dq6 = conduitLossRate<kCold>(p, j, x, dt, &evapRate, &seepRate, ct) * 2.5 * dt * v / len0;
    } else {
        // the loss rate is 0: ((0 * 2.5) * dt * v) / len0 with dt, len0 > 0
        // finite is exactly 0 * v (a signed zero, or NaN for a non-finite v,
        // as in dwflow.c:236) -- without the division
        dq6 = 0.0 * v;
    }

    double denom = 1.0 + dq1 + dq5;
    double rDh, rDl;                                   // rDh = 1.0 / denom
    recipDDFast(denom, &rDh, &rDl);
    double q = divDD(qOld - dq2 + dq3 + dq4 + dq6, denom, rDh, rDl);
    double dqdhV = divDD(rDh * 32.2 * dt * aWtd, length, rLh, rLl) * barrels;

    int normalFlow = 0, inletCtl = 0;
    const int culvert = kCold ? (int)((f >> LF_CULVERT_SHIFT) & 0x3F) : 0;
    if (q > 0.0) {
        if (kCold && culvert > 0 && !isFull) {                  // dwflow.c:250-252
            double dq = 0.0;
            q = culvertInflow(x, culvert, p.slope[j], q, h1 - z1, &dq, &inletCtl, ct);
            if (inletCtl) dqdhV = dq;
        } else
        if (p.normalFlowLtd != NFL_NEITHER && y1 < x.yFull && (fc == F_SUBCRIT || fc == F_SUPCRIT)) {
            // checkNormalFlow dwflow.c:637-686
            bool hasOutfall = (f & (LF_N1_OUTFALL | LF_N2_OUTFALL)) != 0;
            bool check = false;
            if (p.normalFlowLtd == NFL_SLOPE || p.normalFlowLtd == NFL_BOTH || hasOutfall)
                if (y1 < y2) check = true;
            if (!check && (p.normalFlowLtd == NFL_FROUDE || p.normalFlowLtd == NFL_BOTH) && !hasOutfall) {
                if (y1 > 0.0001 && y2 > 0.0001) {
                    double f1;
                    if constexpr (kFast) f1 = circFroude(p, x, q / a1, y1, nd1, c1, a1, w1F, ct);
                    else f1 = linkFroude<kCold>(x, q / a1, y1, ct);
                    if (f1 >= 1.0) check = true;
                }
            }
            if (check) {
                double qNorm = p.beta[j] * a1 * (kFast ? swxPowTwoThirds(r1) : pow(r1, 2. / 3.));
                if (qNorm < q) {
                    normalFlow = 1;
                    q = qNorm;
                }
            }
        }
    }

    if (steps > 0) {
        q = (1.0 - omega) * qLast + omega * q;
        if (q * qLast < 0.0) q = 0.001 * gsgn(q);
    }
    if (f & LF_QLIMIT) {
        double ql = kFast ? p.rare->qLimit[j] : p.qLimit[j];
        if (fabs(q) > ql) q = gsgn(q) * ql;
    }
    // link_setFlapGate (link.c:643-670)
    {
        bool closed = false;
        if (f & LF_FLAP) {
            double dir = (f & LF_DIRNEG) ? -1.0 : 1.0;
            if (q * dir < 0.0) closed = true;
        }
        if (!closed) {
            if (q < 0.0 && (f & LF_N2_OFLAP)) closed = true;
            if (q > 0.0 && (f & LF_N1_OFLAP)) closed = true;
        }
        if (closed) q = 0.0;
    }
    if (q > 0.0001 && yn1 <= 0.0001) q = 0.0001;
    if (q < -0.0001 && yn2 <= 0.0001) q = -0.0001;

    p.dqdh[j] = dqdhV;
    p.a1[j] = aMid;
    p.q1[j] = q;
    p.lNewDepth[j] = gmin(yMid, x.yFull);
    double aAvg = (a1 + a2) / 2.0;
    int fs = 0;
    if (a1 >= x.aFull) fs = (a2 >= x.aFull) ? FS_ALL_FULL : FS_UP_FULL;
    else if (a2 >= x.aFull) fs = FS_DN_FULL;
    p.lNewVolume[j] = aAvg * len0 * barrels;
    p.lNewFlow[j] = q * barrels;
    if (f & LF_SEEP) {
        if constexpr (kFast) {
            p.rare->evapLoss[j] = evapRate;
            p.rare->seepLoss[j] = seepRate;
        } else {
            p.evapLoss[j] = evapRate;
            p.seepLoss[j] = seepRate;
        }
    }
    int old = p.lstate[j];
    p.lstate[j] = (old & (1 << 9)) | fc | (fs << 4) | (normalFlow << 8) | (inletCtl << 10);
}

// ===========================================================================
//  kernels
// ===========================================================================
__device__ __forceinline__ void stageTables(double* ct, const double* g, int nGeom = 0)
{
    const int n = 5 * SWX_CIRC_N + kGeomVals * nGeom;
    for (int i = threadIdx.x; i < n; i += blockDim.x) ct[i] = g[i];
    __syncthreads();
}

// The step converged at iteration m (dynwave.c:249-251): the frozen junctions
// take their depth at that last iteration (a step that runs all MaxTrials
// iterations does this in its last node update).  Run by the first launch
// after convergence.
__device__ __forceinline__ void finalizeFrozen(const Params& p, int m, int tid, int nthr)
{
    // a node frozen at iteration k >= 1 carries frz = k + 1 >= 2, and
    // frozenDepth advances it over iterations frz - 1 .. m - 1: after a step
    // that converged at iteration m <= 1 no depth moves, and the flags are
    // reset by the next step's iteration-0 node pass (nodePass<true>)
    if (m <= 1) return;
    for (int i = tid; i < p.nN; i += nthr) {
        const int fz = p.frz[i];
        if (fz) {
            p.nNewDepth[i] = frozenDepth(p, i, fz, m);
            p.frz[i] = 0;
        }
    }
}
// iterations run in this step (dynwave.c:242-257), from the per-iteration flags
__device__ __forceinline__ int stepIterations(const Params& p, bool* converged)
{
    if (p.maxTrials <= 1) { *converged = false; return p.maxTrials < 1 ? 0 : 1; }
    // the same scan (while (steps < MaxTrials && unconv[steps - 1]) steps++)
    // over flags loaded eight at a time: the first iteration m >= 1 whose
    // nodes all converged ends the step after m + 1 iterations.  (One flag
    // at a time was a chain of dependent loads at the start of the kernels.)
    for (int base = 1; base < p.maxTrials; base += 8) {
        int f[8];
#pragma unroll
        for (int q = 0; q < 8; q++) f[q] = (base + q < p.maxTrials) ? p.unconv[base + q] : 1;
#pragma unroll
        for (int q = 0; q < 8; q++)
            if (f[q] == 0) { *converged = true; return base + q + 1; }
    }
    *converged = false;
    return p.maxTrials;
}


// XCD-aware block order for the node passes (cdna_hip_programming.md §5.5
// T1): workgroups are dealt round-robin over the 8 XCDs, so block b runs the
// (b % 8)-th eighth of the logical blocks and each XCD sweeps one contiguous
// node range per grid-stride round (a node's links, gathered by both end
// nodes, then mostly meet in one L2).  Speed only: any placement gives the
// same results (each index is still taken by exactly one thread).  Measured
// on the surcharged 1M grid: k_node(0) 40.2 -> 38.5 us, k_node(1) 34.9 ->
// 32.3 us; the streaming k_link (+1.7 us), k_step_end (+6 us) and
// k_qual_node (+0.7 us) were slower with it and keep the plain order.
__device__ __forceinline__ int xcdBlock()
{
    const int g = (int)gridDim.x, b = (int)blockIdx.x;
    if (g & 7) return b;
    return (b & 7) * (g >> 3) + (b >> 3);
}

// measurement only: thread 0 stamps the wall clock into probe slot `slot` of
// iteration k
// (per workgroup: no atomics, whose serialisation would be what is measured;
// the host takes the minimum or maximum over the workgroups)
__device__ __forceinline__ void probeMark(const Params& p, int k, int slot, unsigned who = 0)
{
    if (p.probe && threadIdx.x == who && blockIdx.x < (unsigned)p.probeBlocks)
        p.probe[((size_t)kProbeSlots * k + slot) * p.probeBlocks + blockIdx.x] = (unsigned long long)wall_clock64();
}

// Iterations k >= 2: a conduit is updated unless both end nodes have
// converged (findBypassedLinks dynwave.c:335-345), i.e. exactly the conduits
// incident to the nodes the node update listed as unconverged in the previous
// iteration (outfalls are always listed).  Four threads per listed node walk
// its CSR row, whose bounds came with the list entry; a conduit whose ends
// are both listed is taken by the lower-numbered end.  cnt = the number of
// listed nodes; ct = staged tables.
// (u0, rb0): thread tid's first entry, loaded by the caller ahead of staging
// kWake (k_sparse): a frozen end node of an updated conduit is put on the
// iteration's wake list (once: wmark), since the sparse node phase visits
// only listed nodes; wcnt = the list's length (LDS)
// Append i (where `me`) with its CSR row bounds to a list: one atomic per
// wave.  (Per-chunk segments without atomics were measured slower on the
// surcharged 1M grid: its unconverged nodes are clustered, so the adds are
// few, and the walk over segments could not pack them as tightly.)
__device__ __forceinline__ void waveAppend(bool me, int i, int2 row, int* count, int* list, int2* rows)
{
    unsigned long long m = __ballot(me);
    if (m) {
        int lane = threadIdx.x & 63, leader = __ffsll((long long)m) - 1, base = 0;
        if (lane == leader) base = atomicAdd(count, __popcll(m));
        base = __shfl(base, leader, 64);
        if (me) {
            const int e = base + __popcll(m & ((1ull << lane) - 1ull));
            list[e] = i;
            if (rows) rows[e] = row;
        }
    }
}

// A list under construction: its global count, entries and (optional) row
// bounds, and optionally a workgroup buffer in LDS.  With the buffer a wave
// claims its slots with one LDS atomic and the workgroup flushes once at the
// end (one global atomic per workgroup and list, coalesced copies): per-wave
// global atomics on one counter serialise (about 100 per microsecond), and
// with tens of thousands of nodes appended per iteration that was the list
// kernels' long pole.  Entries past the buffer go straight to the global
// list.  Without the buffer (lds == nullptr) every append is waveAppend (the
// count may itself live in LDS: k_sparse).
// (kCap: the buffer's entries)
constexpr int kLdsListCap = 512;
template <bool kRows, int kCap = kLdsListCap>
struct LdsList {
    int n;
    int idx[kCap];
    int2 row[kRows ? kCap : 1];
};
template <bool kRows, int kCap = kLdsListCap>
struct ListSink {
    int* count;
    int* list;
    int2* rows;
    LdsList<kRows, kCap>* lds;
};
template <bool kRows>
__device__ __forceinline__ ListSink<kRows> directSink(int* count, int* list, int2* rows = nullptr)
{
    return ListSink<kRows>{count, list, rows, nullptr};
}
// workgroup-collective: before the first append (a barrier follows before use)
template <bool kRows, int kCap>
__device__ __forceinline__ void sinkInit(const ListSink<kRows, kCap>& s)
{
    if (s.lds && threadIdx.x == 0) s.lds->n = 0;
}
template <bool kRows, int kCap>
__device__ __forceinline__ void sinkAppend(const ListSink<kRows, kCap>& s, bool me, int i, int2 row)
{
    if (!s.lds) {
        waveAppend(me, i, row, s.count, s.list, kRows ? s.rows : (int2*)nullptr);
        return;
    }
    const unsigned long long m = __ballot(me);
    if (!m) return;
    const int lane = threadIdx.x & 63, leader = __ffsll((long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(&s.lds->n, __popcll(m));
    base = __shfl(base, leader, 64);
    const int e = base + __popcll(m & ((1ull << lane) - 1ull));
    const bool fits = e < kCap;
    if (me && fits) {
        s.lds->idx[e] = i;
        if (kRows) s.lds->row[e] = row;
    }
    waveAppend(me && !fits, i, row, s.count, s.list, kRows ? s.rows : (int2*)nullptr);
}
// workgroup-collective, after the last append; gbase: an LDS int
template <bool kRows, int kCap>
__device__ __forceinline__ void sinkFlush(const ListSink<kRows, kCap>& s, int* gbase)
{
    if (!s.lds) return;
    __syncthreads();
    const int n = (s.lds->n < kCap) ? s.lds->n : kCap;
    if (threadIdx.x == 0) *gbase = n ? atomicAdd(s.count, n) : 0;
    __syncthreads();
    const int b = *gbase;
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
        const int i = s.lds->idx[e];
        s.list[b + e] = i;
        if (kRows) s.rows[b + e] = s.lds->row[e];
    }
}

// (wmark deduplicates the nodes)
__device__ __forceinline__ void sparseWake(const Params& p, bool f1, int n1, bool f2, int n2,
                                           const ListSink<false>& w)
{
    const bool w1 = f1 && atomicExch(&p.wmark[n1], 1) == 0;
    const bool w2 = f2 && atomicExch(&p.wmark[n2], 1) == 0;
    sinkAppend(w, w1, n1, make_int2(0, 0));
    sinkAppend(w, w2, n2, make_int2(0, 0));
}
// skipOut: the conduits with an outfall end are left to deferredOutfalls
template <bool kFast, bool kWake = false>
__device__ __forceinline__ int linkListWalk(const Params& p, int k, int cnt, double dt, const double* ct,
                                            int tid, int nthr, int u0, int2 rb0,
                                            const ListSink<false>& wake = ListSink<false>{},
                                            bool skipOut = false)
{
    const uint32_t skip = LF_COLD | (skipOut ? (LF_N1_OUTFALL | LF_N2_OUTFALL) : 0u);
    const int* list = p.ulist + (size_t)((k - 1) & 1) * p.nN;
    const int2* rows = p.ulistRow + (size_t)((k - 1) & 1) * p.nN;
    const int slots = 4 * cnt;
    int work = 0;
    for (int t = tid; t < slots; t += nthr) {
        const int u = (t == tid) ? u0 : list[t >> 2];
        const int2 rb = (t == tid) ? rb0 : rows[t >> 2];
        for (int e = rb.x + (t & 3); e < rb.y; e += 4) {
            // the entry names the link and (csrOther) its other end, so the
            // end nodes' state loads in parallel with the link's own; the
            // filters' operands and both end depths load together
            const int ent = p.csr[e], o = p.csrOther[e];
            const int l = ent & 0x7FFFFFFF;
            if (o < 0) continue;                      // a ghost link (multi-GPU): its owner updates it
            const int2 nn = (ent < 0) ? make_int2(o, u) : make_int2(u, o);
            const uint32_t f = p.lflags[l];
            const int f1 = p.frz[nn.x], f2 = p.frz[nn.y];
            const int cv = p.conv[o];
            const double d1 = p.nNewDepth[nn.x], d2 = p.nNewDepth[nn.y];
            const double r1 = p.yRaw[nn.x], r2 = p.yRaw[nn.y];
            if (f & skip) continue;                   // the cold conduits' loop (and see skipOut)
            if (!cv && o < u) continue;               // listed too: o takes it
            double y1 = frozenDepthV(d1, r1, f1, k - 1);
            double y2 = frozenDepthV(d2, r2, f2, k - 1);
            conduitFlow<false, false, kFast>(p, l, f, nn, k, dt, ct, y1, y2);
            p.dirty[nn.x] = 1;                        // their sums are stale
            p.dirty[nn.y] = 1;
            if (kWake) sparseWake(p, f1 != 0, nn.x, f2 != 0, nn.y, wake);
            if (p.countWork) atomicAdd(&p.nodeLinkWork[nn.x], 1u);   // measurement only
            work++;
        }
    }
    return work;
}

// kProbe: a separately named instantiation for swmmx_timeKernel's
// back-to-back measurement launches (same code)
template <bool kFirst, int kWaves, bool kFast, bool kProbe = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kWaves)))
void k_link(Params p, int k)
{
    const int tid = blockIdx.x * kBlock + threadIdx.x, nthr = gridDim.x * kBlock;
    const int cnt = (!kFirst && k >= 2) ? p.ucount[k - 1] : 0;   // loads with the flag below
    if (k < 2 && stepIsSteady(p)) return;            // SKIP_STEADY_STATE: no flow routing this step
    if (k >= 2 && p.unconv[k - 1] == 0) {            // converged: dynwave.c:249-251
        // the first launch after the step converged (iteration k-1 ran)
        if (p.freeze && (k == 2 || p.unconv[k - 2] != 0)) finalizeFrozen(p, k - 1, tid, nthr);
        return;
    }
    __shared__ double ct[kFast ? kCtFast : 5 * SWX_CIRC_N];
    probeMark(p, k, PR_L_IN);
    double dt = p.ctl->dt;
    int work = 0;
    if (kFirst && blockIdx.x == 0)
        for (int t = threadIdx.x; t < p.maxTrials; t += kBlock) {
            p.ucount[t] = 0; p.vcount[t] = 0; p.wcount[t] = 0;
            if (p.xwcount) p.xwcount[t] = 0;
        }
    if (kFirst && blockIdx.x == 0 && threadIdx.x == 0) p.ctl->tailBar = 0;
    if (kFirst || k < 2) {
        stageTables(ct, p.gTables, kFast ? p.nGeom : 0);
        for (int j = tid; j < p.nL; j += nthr) {
            uint32_t f = p.lflags[j];
            if (f & LF_COLD) continue;
            int2 nn = p.lnodes[j];
            conduitFlow<kFirst, false, kFast>(p, j, f, nn, k, dt, ct, p.nNewDepth[nn.x], p.nNewDepth[nn.y]);
        }
    } else {
        if (blockIdx.x * kBlock < 4 * cnt) {                // uniform per block
            int u0 = 0;
            int2 rb0 = make_int2(0, 0);
            if (tid < 4 * cnt) {                             // first entry: loads with the staging
                u0 = p.ulist[(size_t)((k - 1) & 1) * p.nN + (tid >> 2)];
                rb0 = p.ulistRow[(size_t)((k - 1) & 1) * p.nN + (tid >> 2)];
            }
            stageTables(ct, p.gTables, kFast ? p.nGeom : 0);
            probeMark(p, k, PR_L_STAGED);
            work = linkListWalk<kFast>(p, k, cnt, dt, ct, tid, nthr, u0, rb0);
            probeMark(p, k, PR_L_WORK);
        }
    }
    probeMark(p, k, PR_L_OUT);
    // measurement only (eager timing launches, iterations >= 2 where links can
    // be bypassed): one atomic per workgroup after an LDS reduction
    if (k >= 2 && p.countWork) {
        __shared__ int wsum[kBlock / 64];
        for (int off = 32; off > 0; off >>= 1) work += __shfl_down(work, off, 64);
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = work;
        __syncthreads();
        if (threadIdx.x == 0) {
            int t = 0;
            for (int w = 0; w < kBlock / 64; w++) t += wsum[w];
            if (t) atomicAdd(&p.work[k], (unsigned long long)t);
        }
    }
}

// table_lookup (table.c:395-426) and table_tseriesLookup with extend = TRUE
// (table.c:745-804) on (x, y) pairs: first / last value outside the range,
// linear interpolation (tableInterp, storage.h) inside
__device__ double curveLookup(const double* t, int n, double x)
{
    if (n <= 0) return 0.0;
    double x1 = t[0], y1 = t[1];
    if (x <= x1) return y1;
    for (int m = 1; m < n; m++) {
        double x2 = t[2 * m], y2 = t[2 * m + 1];
        if (x <= x2) return tableInterp(x, x1, y1, x2, y2);
        x1 = x2;
        y1 = y2;
    }
    return y1;
}
__device__ double tseriesLookupExt(const double* t, int n, double x)
{
    if (n <= 0) return 0.0;
    if (x < t[0]) return t[1];
    for (int m = 1; m < n; m++)
        if (x <= t[2 * m]) return tableInterp(x, t[2 * m - 2], t[2 * m - 1], t[2 * m], t[2 * m + 1]);
    return t[2 * n - 1];
}
// outfall_setOutletDepth's operands (the conduit's offset at the outfall end,
// the outfall's invert and fixed stage), loaded with the conduit's own
// operands: one memory round before the root finding, none after it
struct OutfallOps {
    double z, inv, fixedStage;
};
__device__ __forceinline__ OutfallOps loadOutfallOps(const Params& p, int o, int j, uint32_t f)
{
    OutfallOps r;
    const double z1 = p.off1[j], z2 = p.off2[j];
    r.z = (f & LF_N2_OUTFALL) ? z2 : z1;          // o is node2 when node2 is an outfall
    r.inv = p.invert[o];
    r.fixedStage = p.fixedStage[o];
    return r;
}
__device__ __forceinline__ double outfallCombine(const Params& p, int i, uint32_t nf, const OutfallOps& a,
                                                 double yNorm, double yCrit)
{
    const double z = a.z;
    int ot = (int)((nf >> NF_OTYPE_SHIFT) & 0x7);
    double inv = a.inv;
    if (ot == O_FREE) return (z > 0.0) ? 0.0 : gmin(yNorm, yCrit);
    if (ot == O_NORMAL) return (z > 0.0) ? 0.0 : yNorm;
    double stage = (ot == O_FIXED) ? a.fixedStage : inv;
    if (ot == O_TIDAL || ot == O_TSERIES) {             // node.c:1446-1459
        const double* t = p.ofTab + p.ofOff[2 * i];
        int n = p.ofOff[2 * i + 1];
        double tEnd = p.ctl->newRoutingTime + 1000.0 * p.ctl->dt;   // NewRoutingTime of this step
        if (ot == O_TIDAL) {
            double currentDate = tEnd / 86400000.0;
            double x = t[0] + (currentDate - floor(currentDate)) * 24.0;
            stage = curveLookup(t, n, x) / p.ucfL;
        } else {
            stage = tseriesLookupExt(t, n, p.startDateTime + tEnd / 86400000.0) / p.ucfL;
        }
    }
    yCrit = gmin(yCrit, yNorm);
    double yNew;
    if (yCrit + z + inv < stage) yNew = stage - inv;
    else if (z > 0.0) {
        if (stage < inv + z) yNew = gmax(0.0, (stage - inv));
        else yNew = z + yCrit;
    } else yNew = yCrit;
    return yNew;
}


// The few conduits with an invert offset or an outfall end (compacted list):
// full flow classification with normal / critical depth.
template <bool kFirst, bool kWake>
__device__ __forceinline__ int coldConduitsS(const Params& p, int k, double dt, const double* ct, int tid, int nthr,
                                             const ListSink<false>& wake)
{
    int work = 0;
    for (int c = tid; c < p.nCold; c += nthr) {
        int j = p.coldLinks[c];
        uint32_t f = p.lflags[j];
        int2 nn = p.lnodes[j];
        if (k >= 2 && p.conv[nn.x] && p.conv[nn.y]) continue;
        const int f1 = (k >= 2) ? p.frz[nn.x] : 0, f2 = (k >= 2) ? p.frz[nn.y] : 0;
        double y1 = frozenDepth(p, nn.x, f1, k - 1);
        double y2 = frozenDepth(p, nn.y, f2, k - 1);
        conduitFlow<kFirst, true>(p, j, f, nn, k, dt, ct, y1, y2);
        if (k >= 2) { p.dirty[nn.x] = 1; p.dirty[nn.y] = 1; }
        if (kWake) sparseWake(p, f1 != 0, nn.x, f2 != 0, nn.y, wake);
        if (k >= 2 && p.countWork) atomicAdd(&p.nodeLinkWork[nn.x], 1u);   // measurement only
        work++;
    }
    return work;
}
template <bool kFirst, bool kWake = false>
__device__ __forceinline__ int coldConduits(const Params& p, int k, double dt, const double* ct, int tid, int nthr,
                                            int* wcnt = nullptr)
{
    return coldConduitsS<kFirst, kWake>(p, k, dt, ct, tid, nthr, directSink<false>(wcnt, p.wlist));
}
// kWake: the list graph's iterations k >= 2 (frozen end nodes of updated
// conduits go on the wake list, wcount[k])
template <bool kFirst, bool kWake = false>
__global__ __launch_bounds__(kBlock) void k_link_cold(Params p, int k)
{
    if (k >= 2 && p.unconv[k - 1] == 0) return;
    if (k < 2 && stepIsSteady(p)) return;            // SKIP_STEADY_STATE
    __shared__ double ct[5 * SWX_CIRC_N];
    stageTables(ct, p.gTables);
    (void)coldConduits<kFirst, kWake>(p, k, p.ctl->dt, ct, blockIdx.x * kBlock + threadIdx.x, gridDim.x * kBlock,
                                      kWake ? &p.wcount[k] : nullptr);
}

// storage unit i's area relation (node_getVolume / node_getSurfArea for
// STORAGE); out of line: only storage nodes call them
__device__ __forceinline__ StorageGeom devStorageGeom(const Params& p, int i)
{
    StorageGeom g;
    g.shape = p.stShape[i];
    g.a0 = p.stA0[i];
    g.a1 = p.stA1[i];
    g.a2 = p.stA2[i];
    int off = p.stCOff[i];
    g.cx = p.curveX + off;
    g.cy = p.curveY + off;
    g.cn = p.stCN[i];
    g.fullDepth = p.fullDepth[i];
    g.fullVolume = p.fullVolume[i];
    g.ucfL = p.ucfL;
    g.ucfV = p.ucfV;
    return g;
}
__device__ __attribute__((noinline)) double devStorageVolume(const Params& p, int i, double d)
{
    return storageVolume(devStorageGeom(p, i), d);
}
__device__ __attribute__((noinline)) double devStorageArea(const Params& p, int i, double d)
{
    return storageSurfArea(devStorageGeom(p, i), d);
}
__device__ __attribute__((noinline)) double devStorageLosses(const Params& p, int i, double depth,
                                                            double volume, double dt, double* evapVol,
                                                            double* exfilVol)
{
    const int x = p.exIdx[i];
    const StepCtl* c = p.ctl;
    return storageLossesEx(devStorageGeom(p, i), p.stFEvap[i], c->evapRate, depth, volume, dt,
                           x >= 0 ? p.exData + (size_t)kExVals * x : nullptr, c->hydconFactor, c->recoveryFactor,
                           evapVol, exfilVol);
}

// A converged plain junction (not surcharged, ponded or flooded, no storage
// volume) whose sums stay unchanged relaxes toward yRaw with a step that
// halves every iteration, so it stays converged; it stays on the plain branch
// when its depth and yRaw both lie in [0, yCrown (EXTRAN)] and [0, yMax]
// (relaxed values lie between them).  Such a junction may be frozen.
__device__ __forceinline__ bool freezable(const Params& p, double yNew, double yRaw, double yMax, double yCrown)
{
    if (!(yRaw >= 0.0) || yNew > yMax || yRaw > yMax) return false;
    if (p.surchargeMethod == SUR_EXTRAN && yCrown > 0.0 && (yNew > yCrown || yRaw > yCrown)) return false;
    return true;
}

// setNodeDepth (dynwave.c:636-762) for node i given its summed inflow,
// outflow, surface area and dq/dh; returns 1 when converged (dynwave.c:615-621)
template <bool kStorage = true>
__device__ __forceinline__ int nodeUpdate(const Params& p, int i, int k, uint32_t nf, double dt,
                                          double yLast, double yOld, double inflow, double outflow,
                                          double surf, double sumdqdh)
{
    const double omega = 0.5;
    bool canPond = (nf & NF_CANPOND) != 0;
    double fullDepth = p.fullDepth[i];
    bool isPonded = (canPond && yLast > fullDepth);
    double yCrown = p.yCrown[i];
    double overflow = 0.0;
    double surfArea = gmax(surf, p.minSurfArea);
    double dQ = inflow - outflow;
    double dV = 0.5 * (p.oldNetInflow[i] + dQ) * dt;
    const bool isStorage = kStorage && (int)(nf & NF_TYPE) == STORAGE;
    bool isSurcharged = false;
    if (p.surchargeMethod == SUR_EXTRAN) {
        if (isPonded) isSurcharged = false;
        else if (isStorage) isSurcharged = (p.surDepth[i] > 0.0 && yLast > fullDepth);
        else isSurcharged = (yCrown > 0.0 && yLast > yCrown);
    }
    double yNew, dy;
    double yRaw = 0.0;
    if (!isSurcharged) {
        dy = dV / surfArea;
        yNew = yOld + dy;
        yRaw = yNew;
        if (!isPonded) p.oldSurfArea[i] = surfArea;
        if (k > 0) yNew = (1.0 - omega) * yLast + omega * yNew;
        if (isPonded && yNew < fullDepth) yNew = fullDepth - 0.0001;
    } else {
        double corr = (nf & NF_DEGNEG) ? 0.6 : 1.0;
        double denom = sumdqdh;
        if (yLast < 1.25 * yCrown) {
            double fr = (yLast - yCrown) / yCrown;
            denom += (p.oldSurfArea[i] / dt - sumdqdh) * exp(-15.0 * fr);
        }
        if (denom == 0.0) dy = 0.0;
        else dy = corr * dQ / denom;
        yNew = yLast + dy;
        if (yNew < yCrown) yNew = yCrown - 0.0001;
        if (canPond && yNew > fullDepth) yNew = fullDepth + 0.0001;
    }
    if (yNew < 0) yNew = 0.0;
    double yMax = fullDepth;
    if (!canPond) yMax += p.surDepth[i];
    double fullVolume = p.fullVolume[i];
    const bool flooded = yNew > yMax;
    const bool plain = !isSurcharged && !canPond && !flooded && fullVolume == 0.0 && !isStorage;
    if (k >= 1) {                                      // fast-path cache for the next iteration
        if (plain) p.yRaw[i] = yRaw;
        p.dirty[i] = plain ? 2 : 0;
    }
    if (flooded) {                                     // getFloodedDepth dynwave.c:766-795
        double newVolume;
        if (!canPond) {
            overflow = dV / dt;
            newVolume = fullVolume;
            yNew = yMax;
        } else {
            double oldVolume = p.nOldVolume[i];
            newVolume = gmax((oldVolume + dV), fullVolume);
            overflow = (newVolume - gmax(oldVolume, fullVolume)) / dt;
        }
        if (overflow < 0.0001) overflow = 0.0;
        p.nNewVolume[i] = newVolume;
    } else if (kStorage && isStorage) {
        p.nNewVolume[i] = devStorageVolume(p, i, yNew);
    } else {
        p.nNewVolume[i] = (fullDepth > 0.0) ? fullVolume * (yNew / fullDepth) : 0.0;
    }
    p.overflow[i] = overflow;
    p.nNewDepth[i] = yNew;     // Xnode.dYdT = |yNew - yOld| / dt: formed at the step end
    int c = (fabs(yLast - yNew) > p.headTol) ? 0 : 1;  // dynwave.c:615-621
    p.conv[i] = c;
    if (k >= 1 && k + 1 < p.maxTrials && p.freeze && plain && c && !(nf & NF_DEFER) &&
        (p.xwake || !(nf & (NF_SHARED | NF_REPLICA))) && freezable(p, yNew, yRaw, yMax, yCrown)) {
        p.frz[i] = (unsigned char)(k + 1);
        return c | 2;                                  // bit 1: frozen by this update
    }
    return c;
}

// kGeneral: the network has storage units or non-basic conduit shapes.  Their
// area relations are out-of-line calls whose stack frames and registers would
// give every node update a large scratch segment (and throttle its waves), so
// the other networks use a node update without them.
// prologue of the node update: outfall depths (link_setOutfallDepth,
// findNodeDepths dynwave.c:605) from this iteration's link flows, on the
// blocks with blockIdx.x * 64 < nOutLinks, 64 outfall conduits per block and
// round.  Wave 0 finds their normal depths (one lane per conduit; the
// small-flow circular case is an inherently serial Newton solve).  Waves 1-3
// find their critical depths in groups of 32 lanes, one conduit per group:
// the 26 critical flows at getYcritEnum's depth increments (geometry only,
// tabulated at init by k_outfall_qcs) are loaded one per lane and the group's
// first lane runs the enumeration's search on them
// (yCritEnumScan: the same values and operations as the serial search, which
// evaluates up to 25 of them one after another).  Wave 0 then combines.
// ct = staged circular tables; sh = OutfallLds scratch.
struct OutfallLds {
    double yc[64];
    double qcs[6][32];
};
__device__ __forceinline__ int outLinkAt(const Params& p, int c)
{
    // the first four from the kernel arguments: no load before the conduit's own
    if (c < 4) return c == 0 ? p.outInl0 : c == 1 ? p.outInl1 : c == 2 ? p.outInl2 : p.outInl3;
    return p.outLinks[c];
}
__device__ __forceinline__ int outNodeAt(const Params& p, int c)
{
    if (c < 4) return c == 0 ? p.outNd0 : c == 1 ? p.outNd1 : c == 2 ? p.outNd2 : p.outNd3;
    return p.outNodes[c];
}
// link_setOutfallDepth + outfall_setOutletDepth (link.c:728-766,
// node.c:1413-1492): the normal and the critical depth of each outfall
// conduit's flow on different waves, then the outlet depth from both
// (outfallCombine).  stage: the tables are staged into ct here, after the
// first round's operand loads are issued (they then travel together)
struct BlockSync {
    __device__ void operator()() const { __syncthreads(); }
};
// kGroups: 32-lane critical-depth groups on waves 1.. (6 = waves 1-3 of a
// 256-thread block); Sync: the barrier between the team's waves (the whole
// block, or k_sparse's prologue team only)
template <bool kFirst, bool kGeneral, int kGroups = 6, class Sync = BlockSync>
__device__ __forceinline__ void outfallPrologue(const Params& p, const double* ct, OutfallLds* sh, bool stage,
                                                int kProbeK = 0, Sync sync = Sync())
{
    static_assert(kGroups >= 1 && kGroups <= 6, "OutfallLds holds six groups");
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = (threadIdx.x - 64) >> 5, gl = threadIdx.x & 31;    // waves 1-3: 6 groups of 32 lanes
    for (int base = blockIdx.x * 64; base < p.nOutLinks; base += gridDim.x * 64) {
        const int nHere = (p.nOutLinks - base < 64) ? p.nOutLinks - base : 64;
        // wave 0: lane's outfall conduit (normal depth, then the outlet
        // depth); waves 1-3: their group's first conduit (critical depth)
        const int c = (w == 0) ? lane : g;
        const int j = (c < nHere) ? outLinkAt(p, base + c) : -1;
        // every operand in one round: the flag word, the section, the flow,
        // the outfall node's state and the combine's operands
        const uint32_t f = (j >= 0) ? p.lflags[j] : 0u;
        Geom x = {};
        double q = 0.0, qMax = 0.0, beta = 0.0;
        int o = -1;
        double prev = 0.0;
        uint32_t nfo = 0;
        OutfallOps ops{0.0, 0.0, 0.0};
        if (j >= 0) {
            x = loadGeomEager(p, j, f);
            q = p.lNewFlow[j];
            if (w == 0) {                              // the outlet node's operands
                qMax = p.qMax[j];
                beta = p.beta[j];
                o = outNodeAt(p, base + c);            // link.c:743-753 (node2 first)
                prev = p.nNewDepth[o];
                nfo = p.nflags[o];
                ops = loadOutfallOps(p, o, j, f);
            }
        }
        const bool cond = (j >= 0) && !(f & LF_NC);
        if (cond) q = fabs(q / (double)((f >> LF_BARREL_SHIFT) & 0xFF));
        // the group's first conduit's tabulated critical flows (static)
        const double qcs0 = (w >= 1 && g < nHere && gl <= 25) ? p.ofQcs[26 * (base + g) + gl] : 0.0;
        if (stage) { stageTables(const_cast<double*>(ct), p.gTables); stage = false; }
        if (base == 0) probeMark(p, kProbeK, PR_P_STAGED);
        double yn = 0.0;                               // non-conduits: yNorm = yCrit = 0
        if (w == 0 && cond) yn = linkYnorm<kGeneral>(x, q, qMax, beta, ct);
        if (base == 0) probeMark(p, kProbeK, PR_P_YN);
        if (w >= 1) {
            for (int m = g; m < nHere; m += kGroups) {
                uint32_t ff = f;
                double qq = q;
                Geom xx = x;
                bool cc = cond;
                if (m != g) {                          // later conduits of the group
                    const int jj = outLinkAt(p, base + m);
                    ff = p.lflags[jj];
                    cc = !(ff & LF_NC);
                    if (cc) {
                        xx = loadGeomEager(p, jj, ff);
                        qq = fabs(p.lNewFlow[jj] /
                                  (double)((ff >> LF_BARREL_SHIFT) & 0xFF));
                    }
                }
                double ycv = 0.0;
                if (cc) {
                    double y0 = 0.0;
                    if (yCritByEnum(xx, qq, &y0)) {
                        if (gl <= 25) sh->qcs[g][gl] = (m == g) ? qcs0 : p.ofQcs[26 * (base + m) + gl];
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        if (gl == 0) ycv = gmin(yCritEnumScan(xx, qq, y0, sh->qcs[g]), xx.yFull);
                        __builtin_amdgcn_wave_barrier();
                    } else if (gl == 0) {
                        ycv = getYcrit<kGeneral>(xx, qq, ct);
                    }
                }
                if (gl == 0) sh->yc[m] = ycv;
            }
            if (base == 0) probeMark(p, kProbeK, PR_P_YC, 64);
        }
        sync();
        if (j >= 0 && w == 0) {
            if (kFirst) p.nOldDepth[o] = prev;             // node_setOldHydState before the update
            if (p.nNC) p.nPrevDepth[o] = prev;
            const double yo = outfallCombine(p, o, nfo, ops, yn, sh->yc[lane]);
            p.nNewDepth[o] = yo;
        }
        sync();
    }
}

// end of a node pass: the iteration's convergence flag (one per iteration;
// any writer stores 1, no atomics needed; all-reduced over the ranks) and the
// measurement counters
__device__ __forceinline__ void nodePassEnd(const Params& p, int k, bool anyUnconv, int gathered, int live, int fast,
                                            bool counted)
{
    if (__any(anyUnconv) && (threadIdx.x & 63) == 0) p.unconv[k] = 1;
    if (counted && p.countWork) {                          // measurement only
        for (int off = 32; off > 0; off >>= 1) {
            gathered += __shfl_down(gathered, off, 64);
            live += __shfl_down(live, off, 64);
            fast += __shfl_down(fast, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            if (gathered) atomicAdd(&p.work[p.maxTrials + k], (unsigned long long)gathered);
            if (live) atomicAdd(&p.work[2 * p.maxTrials + k], (unsigned long long)live);
            if (fast) atomicAdd(&p.work[3 * p.maxTrials + k], (unsigned long long)fast);
        }
    }
}

// One node of findNodeDepths (dynwave.c:593-626) at iteration k: the
// frozen-junction and relaxation shortcuts (k >= 2), the CSR gather and
// setNodeDepth.  listMe: unconverged after this iteration (outfalls always);
// row: its CSR row bounds for the next link walk.  gathered / live / fast:
// measurement counters (countWork).
// a node's flag words, loaded ahead of its update (NodePre)
struct NodePre {
    uint32_t nf;
    unsigned char cache;      // dirty[i] (iterations k >= 2)
    unsigned char fz;         // frz[i] (iterations k >= 2)
};
__device__ __forceinline__ NodePre loadNodePre(const Params& p, int i, int k)
{
    NodePre q{0u, 0, 0};
    if ((unsigned)i < (unsigned)p.nN) {
        q.nf = p.nflags[i];
        if (k >= 2) {
            q.cache = p.dirty[i];
            q.fz = p.frz[i];
        }
    }
    return q;
}

// alive: not frozen after this iteration (k_sparse's live list)
// rowIn: the node's CSR row bounds when its list entry carries them (x < 0:
// load them)
// where a node's gather reads its row and its links' values
struct GatherSrc {
    const int* csr;
    const double *q, *sa1, *sa2, *dqdh, *evap, *seep;
    const uint32_t* lf;
};
__device__ __forceinline__ GatherSrc gatherSrcOf(const Params& p)
{
    return GatherSrc{p.csr, p.lNewFlow, p.sa1, p.sa2, p.dqdh, p.evapLoss, p.seepLoss, p.lflags};
}
template <bool kFirst, bool kGeneral>
__device__ __forceinline__ void nodeItem(const Params& p, int k, int i, double dt, NodePre pre, bool& listMe,
                                         int2& row, bool& anyUnconv, int& gathered, int& live, int& fast,
                                         bool& alive, int2 rowIn = make_int2(-1, -1))
{
    constexpr bool kStorage = kGeneral;
    const GatherSrc gs = gatherSrcOf(p);
        const uint32_t nf = pre.nf;
        int type = (int)(nf & NF_TYPE);
        // an outfall's depth is written by the prologue above: not read here
        double yLast = 0.0;
        bool haveYLast = false;
        listMe = (type == OUTFALL);
        alive = true;
        bool done = false, isFast = false;
        if (!kFirst && k >= 2) {
            const unsigned char cache = pre.cache;
            const int fz = pre.fz;
            if (fz) {
                // frozen junction: nothing to do while its conduits are
                // bypassed (it stays converged; none of its operands is
                // read); once one is updated it is live again from its
                // depth at the last iteration
                if (cache & 1) {
                    yLast = frozenDepth(p, i, fz, k - 1);
                    haveYLast = true;
                    p.frz[i] = (unsigned char)0;
                } else {
                    if (k == p.maxTrials - 1) {            // the last possible iteration
                        p.nNewDepth[i] = frozenDepth(p, i, fz, k);
                        p.frz[i] = (unsigned char)0;
                    }
                    alive = false;
                    done = true;
                }
            } else if (type != OUTFALL && !(nf & NF_DEFER) && (p.xwake || !(nf & NF_SHARED)) && cache == 2) {
                // plain clean junction: the relaxation step of setNodeDepth
                // (dynwave.c:700-715) on the cached unrelaxed depth
                double yLast2 = p.nNewDepth[i], yCrown = p.yCrown[i], yRaw = p.yRaw[i],
                       yMax = p.yMaxNP[i];
                row = (rowIn.x >= 0) ? rowIn : make_int2(p.rowptr[i], p.rowptr[i + 1]);
                bool sur = p.surchargeMethod == SUR_EXTRAN && yCrown > 0.0 && yLast2 > yCrown;
                if (!sur) {
                    const double omega = 0.5;
                    double yNew = (1.0 - omega) * yLast2 + omega * yRaw;
                    if (yNew < 0) yNew = 0.0;
                    if (!(yNew > yMax)) {
                        p.nNewDepth[i] = yNew;
                        int c = (fabs(yLast2 - yNew) > p.headTol) ? 0 : 1;
                        p.conv[i] = c;
                        if (!c) { anyUnconv = true; listMe = true; }
                        else if (p.freeze && k + 1 < p.maxTrials && freezable(p, yNew, yRaw, yMax, yCrown)) {
                            p.frz[i] = (unsigned char)(k + 1);
                            alive = false;
                        }
                        done = true;
                        isFast = true;
                    }
                }
            }
        }
        if (!done || isFast) {
            live++;
            if (!kFirst && k >= 2 && p.countWork) p.nodeWork[i] += 1u;   // (one thread per node and launch)
        }
        if (isFast) fast++;
        if (!done) {
        // the CSR row bounds load with the node's own state (not after the
        // reuse test): one dependent round trip fewer before the gather
        const int e0 = (rowIn.x >= 0) ? rowIn.x : p.rowptr[i], e1 = (rowIn.x >= 0) ? rowIn.y : p.rowptr[i + 1];
        row = make_int2(e0, e1);
        if (!haveYLast) yLast = (type == OUTFALL) ? 0.0 : p.nNewDepth[i];
        double yOld, lat;
        if (kFirst) {
            // routing.c:328-332, node.c:293-304, 325-341 -- step-begin rotation
            double inflowPrev = p.inflow[i], outflowPrev = p.outflow[i];
            yOld = yLast;
            if (type != OUTFALL) p.nOldDepth[i] = yOld;   // outfalls: rotated in the prologue
            p.nOldVolume[i] = p.nNewVolume[i];
            p.oldFlowInflow[i] = inflowPrev;
            p.oldNetInflow[i] = inflowPrev - outflowPrev;
            p.oldLat[i] = p.newLat[i];
            lat = p.latIn[i];
            p.newLat[i] = lat;
            if (kStorage && type == STORAGE) {       // addSystemInflows: node_getLosses (routing.c:363-365)
                double ev = 0.0, xv = 0.0;
                p.nLosses[i] = devStorageLosses(p, i, yOld, p.nOldVolume[i], p.ctl->dt, &ev, &xv);
                p.nEvapVol[i] = ev;
                p.nExfilVol[i] = xv;
            }
        } else {
            yOld = p.nOldDepth[i];
            lat = p.newLat[i];
        }
        double inflow, outflow, surf, sumdqdh;
        const bool reuse = !kFirst && k >= 2 && !(nf & (NF_CANPOND | NF_DEFER)) &&
                           (p.xwake || !(nf & NF_SHARED)) && type != STORAGE && !(pre.cache & 1);
        if (reuse) {
            inflow = p.inflow[i];
            outflow = p.outflow[i];
            surf = p.nSurf[i];
            sumdqdh = p.nDqdh[i];
        } else {
            // initNodeStates (dynwave.c:297-331)
            bool canPond = (nf & NF_CANPOND) != 0;
            double fullDepth = p.fullDepth[i];
            surf = 0.0;
            if (canPond && yLast > fullDepth) surf = p.pondedArea[i];
            inflow = 0.0;
            outflow = 0.0;                        // node losses are 0 for non-storage nodes
            if (kStorage && type == STORAGE) {
                surf = devStorageArea(p, i, yLast);
                outflow = p.nLosses[i];
            }
            if (lat >= 0.0) inflow += lat;
            else outflow -= lat;
            sumdqdh = 0.0;
            // one entry's terms, in updateNodeFlows' order (lossSum: its
            // evaporation + seepage rate, read only for LF_SEEP links)
            auto addEntry = [&](int ent, double q, uint32_t lf, double sav, double dqv, double lossSum) {
                const bool isN2 = ent < 0;
                double barrels = (double)((lf >> LF_BARREL_SHIFT) & 0xFF);
                if (!isN2) {
                    if (q >= 0.0) outflow += q; else inflow -= q;
                } else {
                    if (q >= 0.0) inflow += q; else outflow -= q;
                }
                if (lf & LF_SEEP) {
                    double lossRate = lossSum * barrels;
                    if (lossRate > 0.0) {
                        bool o1 = (lf & LF_N1_OUTFALL) != 0, o2 = (lf & LF_N2_OUTFALL) != 0;
                        if (!o1 && !o2) lossRate /= 2.0;
                        if (!isN2 && !o1) outflow += lossRate;
                        if (isN2 && !o2) outflow += lossRate;
                    }
                }
                surf += sav * barrels;
                sumdqdh += dqv;
            };
            // CSR gather in link-index order == updateNodeFlows serial order,
            // kGather entries at a time: their CSR words, then all their link
            // values, are loaded together before the in-order sums (a row
            // walked one entry at a time is two dependent loads per entry)
            constexpr int kGather = 4;
            for (int eb = e0; eb < e1; eb += kGather) {
                int ent[kGather];
                double qv[kGather], sav[kGather], dqv[kGather];
                uint32_t lfv[kGather];
#pragma unroll
                for (int t = 0; t < kGather; t++)
                    ent[t] = (eb + t < e1) ? gs.csr[eb + t] : 0;
#pragma unroll
                for (int t = 0; t < kGather; t++) {
                    if (eb + t < e1) {
                        const int l = ent[t] & 0x7FFFFFFF;
                        qv[t] = gs.q[l];
                        lfv[t] = gs.lf[l];
                        const double* sp = (ent[t] < 0) ? &gs.sa2[l] : &gs.sa1[l];
                        sav[t] = *sp;
                        dqv[t] = gs.dqdh[l];
                    }
                }
#pragma unroll
                for (int t = 0; t < kGather; t++) {
                    if (eb + t >= e1) break;
                    const int l = ent[t] & 0x7FFFFFFF;
                    const double lossSum = (lfv[t] & LF_SEEP) ? (gs.evap[l] + gs.seep[l])
                                                              : 0.0;
                    addEntry(ent[t], qv[t], lfv[t], sav[t], dqv[t], lossSum);
                }
            }
            p.inflow[i] = inflow;
            p.outflow[i] = outflow;
            // (the gather-reuse sums are read by the iterations k >= 2 of this
            // step only)
            p.nSurf[i] = surf;
            p.nDqdh[i] = sumdqdh;
            if (!kFirst && k >= 2) p.dirty[i] = 0;
            gathered++;
        }
        if (type == OUTFALL) {
            // depth set by the prologue
        } else if (nf & NF_DEFER) {
            // conduit sums written above; k_nc adds the non-conduit links
            // and updates the depth
        } else {
            const int r = nodeUpdate<kStorage>(p, i, k, nf, dt, yLast, yOld, inflow, outflow, surf, sumdqdh);
            if (!(r & 1)) {
                anyUnconv = true;
                listMe = true;
            }
            if (r & 2) alive = false;
        }
        }
}

template <bool kFirst, bool kGeneral>
__device__ __forceinline__ void nodePass(const Params& p, int k, int tid, int nthr, NodePre pre0)
{
    const double dt = p.ctl->dt;
    bool anyUnconv = false;
    int gathered = 0, live = 0, fast = 0;          // measurement only (countWork)
    // this iteration's unconverged nodes (the next walk's list) and, after
    // iteration 1, the live nodes: workgroup-buffered appends (ListSink)
    __shared__ LdsList<true> ldsU;
    __shared__ LdsList<true> ldsV;
    __shared__ int sBase;
    const ListSink<true> su{&p.ucount[k], p.ulist + (size_t)(k & 1) * p.nN, p.ulistRow + (size_t)(k & 1) * p.nN,
                            &ldsU};
    const ListSink<true> sv{&p.vcount[1], p.vlist + p.nN, p.vlistRow + p.nN, &ldsV};
    const bool listV = !kFirst && k == 1 && p.buildVlist;
    if (!kFirst) {
        sinkInit(su);
        sinkInit(sv);
        __syncthreads();
    }
    NodePre pre = pre0;
    int alives = 0;                                // k == 1: nodes not frozen (blockLive)
    for (int i = tid; i < p.nN; i += nthr) {
        bool listMe = false;                   // unconverged after this iteration
        int2 row = make_int2(0, 0);            // its CSR row, for the next walk
        // the thread's next node's flag words load ahead of this node's
        // update: a sparse iteration skips most nodes on their flags alone,
        // so a thread's nodes cost one load latency, not one each
        const NodePre preNext = loadNodePre(p, i + nthr, k);
        bool alive = true;
        // a step starts with no frozen node: the flags a step that converged
        // at iteration 1 left (finalizeFrozen) are cleared here
        if (kFirst && p.freeze) p.frz[i] = 0;
        nodeItem<kFirst, kGeneral>(p, k, i, dt, pre, listMe, row, anyUnconv, gathered, live, fast, alive);
        // list this iteration's unconverged nodes for the next k_link
        if (!kFirst) sinkAppend(su, listMe, i, row);
        // after iteration 1: the nodes not frozen, for the list-driven node
        // phases (k_sparse, k_node_list) of the graphs that run them
        if (!kFirst && k == 1) {
            alives += alive ? 1 : 0;
            if (listV) sinkAppend(sv, alive, i, row);
        }
        pre = preNext;
    }
    if (!kFirst) {
        sinkFlush(su, &sBase);
        if (listV) sinkFlush(sv, &sBase);
    }
    if (!kFirst && k == 1) {                       // the workgroup's live count: no atomics
        __shared__ int sAlive;
        if (threadIdx.x == 0) sAlive = 0;
        __syncthreads();
        for (int off = 32; off > 0; off >>= 1) alives += __shfl_down(alives, off, 64);
        if ((threadIdx.x & 63) == 0 && alives) atomicAdd(&sAlive, alives);
        __syncthreads();
        if (threadIdx.x == 0 && blockIdx.x < (unsigned)p.blockLiveN) p.blockLive[blockIdx.x] = sAlive;
    }
    nodePassEnd(p, k, anyUnconv, gathered, live, fast, !kFirst && k >= 2);
}

// SKIP_STEADY_STATE, a step in steady state: initSystemInflows /
// addSystemInflows (routing.c:312-333, 358-365) -- the lateral inflows rotate
// and storage units take their losses at the unchanged depth and volume;
// nothing else of the node state moves (node_setOldHydState runs in routeFlow)
template <bool kGeneral>
__device__ __forceinline__ void steadyNodes(const Params& p, int tid, int nthr)
{
    for (int i = tid; i < p.nN; i += nthr) {
        p.oldLat[i] = p.newLat[i];
        p.newLat[i] = p.latIn[i];
        if (kGeneral && (int)(p.nflags[i] & NF_TYPE) == STORAGE) {
            double ev = 0.0, xv = 0.0;
            p.nLosses[i] = devStorageLosses(p, i, p.nNewDepth[i], p.nNewVolume[i], p.ctl->dt, &ev, &xv);
            p.nEvapVol[i] = ev;
            p.nExfilVol[i] = xv;
        }
    }
}

// SKIP_STEADY_STATE: inflowHasChanged (routing.c:775-808) -- a node's lateral
// inflow (this step's against the last one), or an outfall's or terminal
// node's inflow (against the one before the last routed step), changed by
// more than LAT_FLOW_TOL.  Any such node marks StepCtl::steadyChanged (reset
// by k_finalize), which with steadyOk decides the step (stepIsSteady).
__device__ __forceinline__ bool flowChanged(double qOld, double qNew, double tol)
{
    double diff;
    if (fabs(qOld) > 1e-6) diff = (qNew / qOld) - 1.0;            // TINY (consts.h)
    else if (fabs(qNew) > 1e-6) diff = 1.0;
    else diff = 0.0;
    return fabs(diff) > tol;
}
// A pump whose on / off depth its inlet node has crossed gets a new setting
// this step (evaluateControlRules' link_setTargetSetting, routing.c:269-296,
// link.c:604-640): actionCount > 0, never steady (routing.c:388-391).  The
// switch itself is made by k_nc<true> as in every routed step.
__global__ __launch_bounds__(kBlock) void k_steady(Params p)
{
    if (!p.ctl->steadyOk) return;                  // the step routes flow anyway
    bool changed = false;
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < p.nN; i += gridDim.x * kBlock) {
        changed = changed || flowChanged(p.newLat[i], p.latIn[i], p.latFlowTol);
        const uint32_t nf = p.nflags[i];
        if ((int)(nf & NF_TYPE) == OUTFALL || (nf & NF_DEG0))
            changed = changed || flowChanged(p.oldFlowInflow[i], p.inflow[i], p.latFlowTol);
    }
    for (int c = blockIdx.x * kBlock + threadIdx.x; c < p.nNC; c += gridDim.x * kBlock) {
        const NcLink& L = p.ncL[c];
        if (L.type != LK_PUMP) continue;
        const int j = p.ncLinks[c];
        const double set = p.setting[j], y1 = p.nNewDepth[p.lnodes[j].x];
        if ((L.yOff > 0.0 && set > 0.0 && y1 < L.yOff) || (L.yOn > 0.0 && set == 0.0 && y1 > L.yOn)) changed = true;
    }
    if (__any(changed) && (threadIdx.x & 63) == 0) {
        p.ctl->steadyChanged = 1;
        p.ctl->steadyIO[6] = 1.0;                  // several ranks: summed over them (launchStep)
    }
}

template <bool kFirst, bool kGeneral, bool kProbe = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kGeneral ? 3 : 4))) void k_node(Params p, int k)
{
    // the first node's flag words load alongside the convergence flag.  With
    // at most 64 outfall links, block 0 runs the outfall prologue only (it is
    // the launch's long pole: serial root finding) and the other blocks take
    // the nodes; xcdBlock() maps block 0 to 0 either way.  With p.deferPro the
    // prologue of iterations 2 <= k < MaxTrials - 1 runs in the next walk
    // (deferredOutfalls) instead
    const bool pro = kFirst || !(p.deferPro && k >= 2 && k < p.maxTrials - 1);
    const bool proOnly = pro && p.nOutLinks > 0 && p.nOutLinks <= 64 && gridDim.x > 1;
    const int nodeBlocks = (int)gridDim.x - (proOnly ? 1 : 0);
    const int tidX = (xcdBlock() - (proOnly ? 1 : 0)) * kBlock + (int)threadIdx.x;
    const NodePre pre0 = loadNodePre(p, tidX, kFirst ? 0 : k);
    if (k >= 2 && p.unconv[k - 1] == 0) return;
    if (k < 2 && stepIsSteady(p)) {
        // SKIP_STEADY_STATE: no flow routing this step (routing.c:239-241);
        // what routing_execute still does per node is initSystemInflows /
        // addSystemInflows' lateral-inflow rotation and node_getLosses
        // (routing.c:312-333, 358-365), from the unchanged state
        if (kFirst) steadyNodes<kGeneral>(p, blockIdx.x * kBlock + threadIdx.x, gridDim.x * kBlock);
        return;
    }
    probeMark(p, k, PR_N_IN);
    probeMark(p, k, PR_N_LAST_IN);
    // prologue: outfall depths (link_setOutfallDepth, findNodeDepths
    // dynwave.c:605) from this iteration's link flows.  Only the outfall's
    // single link reads that depth (next iteration), and this kernel never
    // reads an outfall's depth, so it can run alongside the node updates; it
    // goes first because it is the long (iterative) part of the launch.  The
    // outfall is never "converged" (dynwave.c:281, 340): its link is never
    // bypassed and the depth is refreshed every iteration, as in the reference.
    // 64 outfall conduits per block and round: wave 0 finds their normal
    // depths while wave 1 finds their critical depths, then wave 0 combines.
    // The prologue reads the circular tables from global memory: the small
    // flows an outfall usually carries take the closed-form Newton solves and
    // never touch them, and staging them into LDS (a load round and a
    // barrier) sat in front of the solves
    if (pro && blockIdx.x * 64 < p.nOutLinks) {
        __shared__ OutfallLds sh;
        outfallPrologue<kFirst, kGeneral>(p, p.gTables, &sh, false, k);
        if (blockIdx.x == 0) probeMark(p, k, PR_N_PRO);
        if (proOnly) {
            probeMark(p, k, PR_N_OUT);
            probeMark(p, k, PR_N_B0);
            return;
        }
    }
    nodePass<kFirst, kGeneral>(p, k, tidX, nodeBlocks * kBlock, pre0);
    probeMark(p, k, PR_N_OUT);
    if (blockIdx.x == 0) probeMark(p, k, PR_N_B0);
}

// ---------------------------------------------------------------------------
// k_tail: Picard iterations k >= 2 of one routing step in ONE launch.  The
// unrolled step graph launches a link and a node kernel for every possible
// iteration; those after convergence exit at once but still cost a dispatch
// each (about 5.5 us, 12 of them per step on a network that converges in two
// iterations).  k_tail runs the same per-iteration code (linkListWalk /
// coldConduits, outfallPrologue, nodePass) with a grid barrier between the
// link and node phases, and stops when an iteration converged -- no launch
// at all for the iterations that do not run.  Its workgroups must all be
// resident (grid = CUs x blocks per CU the occupancy admits, host-checked).
//
// Barrier (cdna_hip_programming.md Guideline 16): every wave drains its
// stores, the workgroup meets, lane 0 releases at agent scope and adds to one
// arrival counter (zeroed by k_link<first> each step), polls it relaxed, and
// acquires at agent scope before the workgroup goes on.  Control words
// written inside the launch (unconv, ucount) are read with atomic loads (the
// vector path: the acquire does not refresh the scalar cache).  The spin is
// bounded: a barrier that never completes sets StepCtl::tailErr and the
// launch ends (the step is then reported as failed by the host).
__device__ __forceinline__ bool tailBarrier(const Params& p, unsigned target)
{
    __shared__ int ok;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(&p.ctl->tailBar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // about 1 s at most (an earlier timeout anywhere ends this one at once)
        int good = __hip_atomic_load(&p.ctl->tailErr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
        for (unsigned spins = 0; good &&
             __hip_atomic_load(&p.ctl->tailBar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target;) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1u << 20)) good = 0;
            else if ((spins & 1023) == 0 &&
                     __hip_atomic_load(&p.ctl->tailErr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) good = 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (!good) __hip_atomic_store(&p.ctl->tailErr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = good;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    return ok != 0;
}

template <bool kFast, bool kGeneral>
__global__ __launch_bounds__(kBlock) void k_tail(Params p)
{
    __shared__ double ct[kFast ? kCtFast : 5 * SWX_CIRC_N];
    __shared__ OutfallLds sh;
    const int tid = blockIdx.x * kBlock + threadIdx.x, nthr = gridDim.x * kBlock;
    const double dt = p.ctl->dt;
    unsigned arrivals = 0;
    for (int k = 2; k < p.maxTrials; k++) {
        // dynwave.c:249-251: iteration k-1 converged -- the step is done
        if (__hip_atomic_load(&p.unconv[k - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
            if (p.freeze) finalizeFrozen(p, k - 1, tid, nthr);
            return;
        }
        if (k == 2) stageTables(ct, p.gTables, kFast ? p.nGeom : 0);   // only when an iteration runs
        coldConduits<false>(p, k, dt, ct, tid, nthr);
        const int cnt = __hip_atomic_load(&p.ucount[k - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int u0 = 0;
        int2 rb0 = make_int2(0, 0);
        if (tid < 4 * cnt) {
            u0 = p.ulist[(size_t)((k - 1) & 1) * p.nN + (tid >> 2)];
            rb0 = p.ulistRow[(size_t)((k - 1) & 1) * p.nN + (tid >> 2)];
        }
        (void)linkListWalk<kFast>(p, k, cnt, dt, ct, tid, nthr, u0, rb0);
        arrivals += gridDim.x;
        if (!tailBarrier(p, arrivals)) return;
        // the every-shape root finders (the cold conduits' callees): calling
        // the lean ones would loosen their register budget, and k_node's
        if (blockIdx.x * 64 < p.nOutLinks) outfallPrologue<false, true>(p, ct, &sh, false, k);
        nodePass<false, kGeneral>(p, k, tid, nthr, loadNodePre(p, tid, k));
        arrivals += gridDim.x;
        if (!tailBarrier(p, arrivals)) return;
    }
}

// ---------------------------------------------------------------------------
// k_sparse: Picard iterations k >= 2 of one routing step in ONE workgroup.
// After iteration 1 almost every junction of a large network is frozen
// (converged, plain, relaxing toward its cached depth); what is left is the
// unconverged list (ulist) and the live list (vlist: the nodes not frozen,
// surcharged ones mostly) -- a few thousand nodes on the surcharged 1M grid.
// One workgroup runs every remaining iteration with workgroup barriers only
// (no grid barrier, no XCD coherence question, no launch per iteration):
//
//   link phase   the cold conduits and the unconverged-list walk of
//                k_link(k) (findBypassedLinks dynwave.c:335-345 +
//                dwflow_findConduitFlow); a frozen end node of an updated
//                conduit goes on the wake list (wmark deduplicates)
//   node phase   waves 0-1: the outfall depths (link_setOutfallDepth,
//                dynwave.c:605) from this iteration's flows, with a
//                two-wave barrier of their own; the other waves: nodeItem
//                (findNodeDepths / setNodeDepth dynwave.c:593-762) over the
//                live list of iteration k-1 and the wake list, appending
//                the unconverged nodes (next walk) and the nodes still not
//                frozen (next node phase)
//   end          iteration k's convergence flag; break when it converged
//                (dynwave.c:249-251)
//
// Every node the full-grid k_node(k) would update is on one of the two lists
// (a node not frozen after k-1 is on vlist; a frozen one is updated only
// when an incident conduit was, i.e. woken), and each is updated by the same
// nodeItem code, so results are bitwise those of the unrolled graph.  The
// frozen junctions are advanced to the step's last iteration by k_unfreeze,
// the next kernel.  Host-chosen per step (Router::step) when the live lists
// are short.
constexpr int kSparseBlock = 512;
constexpr int kSparseTeam = 2;       // waves running the outfall prologue
// k_sparse's prologue team barrier: an LDS arrival counter, monotonic within
// the launch (a wave's target is the end of the phase it arrived in)
struct TeamSync {
    int* cnt;
    __device__ void operator()() const
    {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        if ((threadIdx.x & 63) == 0) {
            const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int target = (old / kSparseTeam + 1) * kSparseTeam;
            while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target)
                __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
};

// node phase of a list-driven iteration k >= 2 (k_sparse, k_node_list):
// nodeItem over the live list of iteration k-1 (vc entries), then the wake
// list (wc entries), appending to iteration k's unconverged list (cntU) and
// live list (cntV)
template <bool kGeneral>
__device__ __forceinline__ void listNodePass(const Params& p, int k, double dt, int t0, int nt, int vc, int wc,
                                             const ListSink<true>& su, const ListSink<false>& sv, bool& anyUnconv,
                                             int& gathered, int& live, int& fast)
{
    const int pc = (k - 1) & 1;
    const int* vprev = p.vlist + (size_t)pc * p.nN;
    for (int t = t0; t < vc + wc; t += nt) {
        const bool woken = t >= vc;
        const int i = woken ? p.wlist[t - vc] : vprev[t];
        bool listMe = false, alive = true;
        int2 row = make_int2(0, 0);
        nodeItem<false, kGeneral>(p, k, i, dt, loadNodePre(p, i, k), listMe, row, anyUnconv, gathered, live, fast,
                                  alive);
        if (woken) p.wmark[i] = 0;
        sinkAppend(su, listMe, i, row);
        sinkAppend(sv, alive, i, row);
    }
}

template <bool kFast, bool kGeneral>
__global__ __launch_bounds__(kSparseBlock) void k_sparse(Params p)
{
    __shared__ double ct[kFast ? kCtFast : 5 * SWX_CIRC_N];
    __shared__ OutfallLds sh;
    // per iteration parity c = k & 1: listed (unconverged) count, live count,
    // woken count, "some node did not converge"; team barrier counter
    __shared__ int sU[2], sV[2], sW[2], sUnc[2], sBar;
    const int tid = threadIdx.x;
    if (p.unconv[1] == 0) return;                  // converged at iteration 1: nothing to run
    if (tid == 0) {
        sU[1] = p.ucount[1];
        sV[1] = p.vcount[1];
        sUnc[1] = 1;
        sU[0] = sV[0] = sW[0] = sW[1] = sUnc[0] = 0;
        sBar = 0;
    }
    stageTables(ct, p.gTables, kFast ? p.nGeom : 0);   // (its barrier publishes the counters too)
    const double dt = p.ctl->dt;
    const bool team = p.nOutLinks > 0;
    const int w = tid >> 6;
    const int M = p.maxTrials;
    for (int k = 2; k < M; k++) {
        const int c = k & 1, pc = c ^ 1;
        if (!sUnc[pc]) break;                      // iteration k-1 converged (uniform: LDS)
        const int cnt = sU[pc], vc = sV[pc];
        probeMark(p, k, PR_L_IN);
        // ---- link phase ----------------------------------------------------
        (void)coldConduits<false, true>(p, k, dt, ct, tid, kSparseBlock, &sW[c]);
        int work = 0;                              // streaming conduits updated (measurement)
        {
            const int* list = p.ulist + (size_t)pc * p.nN;
            const int2* rows = p.ulistRow + (size_t)pc * p.nN;
            int u0 = 0;
            int2 rb0 = make_int2(0, 0);
            if (tid < 4 * cnt) { u0 = list[tid >> 2]; rb0 = rows[tid >> 2]; }
            work += linkListWalk<kFast, true>(p, k, cnt, dt, ct, tid, kSparseBlock, u0, rb0,
                                              directSink<false>(&sW[c], p.wlist));
        }
        probeMark(p, k, PR_L_OUT);
        __syncthreads();
        const int wc = sW[c];
        if (tid == 0) { sU[pc] = 0; sV[pc] = 0; sW[pc] = 0; sUnc[pc] = 0; }   // iteration k+1's slots
        probeMark(p, k, PR_N_IN);
        // ---- node phase ----------------------------------------------------
        int gathered = 0, live = 0, fast = 0;
        if (team && w < kSparseTeam) {
            // the every-shape root finders (the cold conduits' callees, as in
            // k_tail): a call from this kernel to the lean ones would give
            // them, and so k_node, this kernel's looser register budget
            outfallPrologue<false, true, 2 * (kSparseTeam - 1), TeamSync>(p, ct, &sh, false, k, TeamSync{&sBar});
            probeMark(p, k, PR_N_PRO);
        } else {
            const int t0 = team ? tid - 64 * kSparseTeam : tid;
            const int nt = team ? kSparseBlock - 64 * kSparseTeam : kSparseBlock;
            bool anyUnconv = false;
            listNodePass<kGeneral>(p, k, dt, t0, nt, vc, wc,
                                   directSink<true>(&sU[c], p.ulist + (size_t)c * p.nN, p.ulistRow + (size_t)c * p.nN),
                                   directSink<false>(&sV[c], p.vlist + (size_t)c * p.nN), anyUnconv, gathered, live,
                                   fast);
            if (__any(anyUnconv) && (threadIdx.x & 63) == 0) sUnc[c] = 1;
        }
        if (p.countWork) {                         // measurement only (eager timing launches)
            for (int off = 32; off > 0; off >>= 1) {
                work += __shfl_down(work, off, 64);
                gathered += __shfl_down(gathered, off, 64);
                live += __shfl_down(live, off, 64);
                fast += __shfl_down(fast, off, 64);
            }
            if ((threadIdx.x & 63) == 0) {
                if (work) atomicAdd(&p.work[k], (unsigned long long)work);
                if (gathered) atomicAdd(&p.work[M + k], (unsigned long long)gathered);
                if (live) atomicAdd(&p.work[2 * M + k], (unsigned long long)live);
                if (fast) atomicAdd(&p.work[3 * M + k], (unsigned long long)fast);
            }
        }
        probeMark(p, k, PR_N_OUT);
        __syncthreads();
        if (tid == 0) {                            // iteration k's results for the step end
            p.ucount[k] = sU[c];
            p.vcount[k] = sV[c];
            if (sUnc[c]) p.unconv[k] = 1;
        }
    }
}

// Deferred outfall depths (p.deferPro): the outfall prologue of iteration
// k_node(k) was the launch's long pole in every sparse iteration (serial root
// finding on one workgroup, ~10 us, while the listed nodes took ~3 us).  Only
// the outfall conduits read an outfall's depth (in the next iteration's link
// update) and no node update reads it (dynwave.c:593-626 skips outfalls'
// setNodeDepth), so iteration k-1's depths can be found at the start of
// k_walk(k), just before the outfall conduits' iteration-k flows that need
// them, overlapping the rest of the walk instead of ending the node launch.
// Block 0 runs both; the walk leaves the outfall conduits to it (skipOut).
// Host conditions (Router init): one rank, no pumps / regulators, 1-64
// outfall conduits, each the only conduit at its outfall, none cold.  The
// order of operations per value is the reference's: prologue(k-1) reads the
// iteration k-1 flows and writes the depths before the iteration-k flows read
// them.  The every-shape root finders (the cold conduits' callees, as in
// k_tail): calling the lean ones would give them, and so k_node, this
// kernel's looser register budget.
template <bool kFast, bool kWake>
__device__ __forceinline__ void deferredOutfalls(const Params& p, int k, double dt, const double* ct,
                                                 OutfallLds* sh, bool runPro, const ListSink<false>& wake)
{
    if (runPro) outfallPrologue<false, true>(p, p.gTables, sh, false, k - 1);   // (ends with a barrier)
    for (int c = threadIdx.x; c < p.nOutLinks; c += kBlock) {
        const int l = outLinkAt(p, c);
        const uint32_t f = p.lflags[l];
        const int2 nn = p.lnodes[l];
        const int f1 = p.frz[nn.x], f2 = p.frz[nn.y];
        const double y1 = frozenDepthV(p.nNewDepth[nn.x], p.yRaw[nn.x], f1, k - 1);
        const double y2 = frozenDepthV(p.nNewDepth[nn.y], p.yRaw[nn.y], f2, k - 1);
        conduitFlow<false, false, kFast>(p, l, f, nn, k, dt, ct, y1, y2);
        p.dirty[nn.x] = 1;
        p.dirty[nn.y] = 1;
        if (kWake) sparseWake(p, f1 != 0, nn.x, f2 != 0, nn.y, wake);
    }
}

// Iterations k >= 2 as list-driven walks.  k_walk(k): the unconverged-list
// walk of k_link(k) (and, with p.deferPro, the deferred outfall work on block
// 0).  kWake (the list graph): the frozen end nodes of updated conduits go on
// the wake list (count wcount[k]; the cold conduits: k_link_cold<false, true>
// on the side stream, as launchIteration forks it), k_node_list(k) then runs
// the outfall prologue (block 0, as k_node, unless deferred) and nodeItem
// over the live list of k-1 and the wake list, and the frozen junctions'
// final depths come from k_unfreeze after the last iteration.  !kWake (the
// unrolled graph with p.deferPro): k_link(k)'s role, k_node(k) follows, and
// the first launch after convergence advances the frozen junctions
// (finalizeFrozen), as k_link does.  Launches after convergence exit at once.
// kDefer (p.deferPro): a separate instantiation, because the prologue's
// calls give the kernel a scratch segment even where they never run (it cost
// the walk ~8 us per launch on the surcharged 1M grid)
template <bool kFast, bool kWake, bool kDefer>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kLinkWavesDefault))) void k_walk(Params p,
                                                                                                      int k)
{
    const int cnt = p.ucount[k - 1];                  // loads with the flag below
    constexpr bool defer = kDefer;
    const bool firstAfter = k == 2 || p.unconv[k - 2] != 0;
    __shared__ OutfallLds sh;
    if (p.unconv[k - 1] == 0) {                       // converged: dynwave.c:249-251
        if (firstAfter) {
            // iteration k-1's outfall depths (its k_node deferred them)
            if (kDefer && k >= 3 && blockIdx.x == 0) outfallPrologue<false, true>(p, p.gTables, &sh, false, k - 1);
            if (!kWake && p.freeze) finalizeFrozen(p, k - 1, blockIdx.x * kBlock + threadIdx.x, gridDim.x * kBlock);
        }
        return;
    }
    // block 0 takes the outfall work when deferred, the others the walk
    const int wb = (int)blockIdx.x - (defer ? 1 : 0);
    const int tid = wb * kBlock + (int)threadIdx.x, nthr = ((int)gridDim.x - (defer ? 1 : 0)) * kBlock;
    // grid-stride loops: a workgroup with no first-round item has none (uniform)
    if (wb >= 0 && wb * kBlock >= 4 * cnt) return;
    __shared__ double ct[kFast ? kCtFast : 5 * SWX_CIRC_N];
    __shared__ LdsList<false> ldsW;                   // the wake list, flushed once (ListSink)
    __shared__ int sBase;
    const ListSink<false> wake{&p.wcount[k], p.wlist, nullptr, kWake ? &ldsW : nullptr};
    if (kWake) sinkInit(wake);                        // (stageTables' barrier follows)
    probeMark(p, k, PR_L_IN);
    const double dt = p.ctl->dt;
    int u0 = 0;
    int2 rb0 = make_int2(0, 0);
    if (wb >= 0 && tid < 4 * cnt) {
        u0 = p.ulist[(size_t)((k - 1) & 1) * p.nN + (tid >> 2)];
        rb0 = p.ulistRow[(size_t)((k - 1) & 1) * p.nN + (tid >> 2)];
    }
    stageTables(ct, p.gTables, kFast ? p.nGeom : 0);
    probeMark(p, k, PR_L_STAGED);
    int work = 0;
    if (kDefer && wb < 0) deferredOutfalls<kFast, kWake>(p, k, dt, ct, &sh, k >= 3, wake);
    else work = linkListWalk<kFast, kWake>(p, k, cnt, dt, ct, tid, nthr, u0, rb0, wake, defer);
    if (kWake) sinkFlush(wake, &sBase);
    probeMark(p, k, PR_L_WORK);
    probeMark(p, k, PR_L_OUT);
    if (p.countWork) {                                // measurement only
        for (int off = 32; off > 0; off >>= 1) work += __shfl_down(work, off, 64);
        if ((threadIdx.x & 63) == 0 && work) atomicAdd(&p.work[k], (unsigned long long)work);
    }
}

// The list graph's node launch of iteration k >= 2.  The nodes k_node(k)
// would update are (dynwave.c:593-626 with the frozen-junction shortcut):
//   A  the nodes not frozen after iteration k-1 -- the live list vlist(k-1)
//      (k_node(1) / this kernel append them), and
//   B  the frozen junctions an updated conduit touched (dirty): every conduit
//      at an unconverged node of k-1 was updated (the walk), so these are
//      the frozen neighbours of the unconverged list ulist(k-1).
// A frozen junction's frz holds the iteration after which it froze + 1, so
// frz in [1, k] marks "frozen before this iteration" -- a node of A that
// freezes during this launch writes k + 1, one woken here writes 0 -- and B
// needs no wake list from the walk (whose atomics cost it ~7 us).  Several
// unconverged nodes can share a frozen neighbour: the first thread to
// exchange the node's stamp takes it.  Items: vc list entries, then four
// threads per unconverged node over its CSR row.  Appends go through LDS
// (ListSink).  Iterations after convergence exit at once.
template <bool kGeneral>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kGeneral ? 3 : 4))) void k_node_list(Params p,
                                                                                                         int k)
{
    const int vc = p.vcount[k - 1], uc = p.ucount[k - 1];   // load with the flag below
    const int xc = p.xwcount ? p.xwcount[k] : 0;             // C: frozen nodes a changed ghost value woke
    if (p.unconv[k - 1] == 0) return;
    probeMark(p, k, PR_N_IN);
    probeMark(p, k, PR_N_LAST_IN);
    const bool pro = !(p.deferPro && k < p.maxTrials - 1);      // else: in k_walk(k + 1)
    const bool proOnly = pro && p.nOutLinks > 0 && p.nOutLinks <= 64 && gridDim.x > 1;
    if (pro && blockIdx.x * 64 < p.nOutLinks) {
        __shared__ OutfallLds sh;
        outfallPrologue<false, kGeneral>(p, p.gTables, &sh, false, k);
        if (blockIdx.x == 0) probeMark(p, k, PR_N_PRO);
        if (proOnly) {
            probeMark(p, k, PR_N_OUT);
            probeMark(p, k, PR_N_B0);
            return;
        }
    }
    const int b = (int)blockIdx.x - (proOnly ? 1 : 0);
    const int nt = ((int)gridDim.x - (proOnly ? 1 : 0)) * kBlock;
    const int items = vc + 4 * uc + xc;
    // a workgroup with no first-round item has none (uniform)
    if (b * kBlock >= items) return;
    __shared__ LdsList<true> ldsU;
    __shared__ LdsList<true> ldsV;
    __shared__ int sBase;
    const int c = k & 1, pc = c ^ 1;
    const ListSink<true> su{&p.ucount[k], p.ulist + (size_t)c * p.nN, p.ulistRow + (size_t)c * p.nN, &ldsU};
    const ListSink<true> sv{&p.vcount[k], p.vlist + (size_t)c * p.nN, p.vlistRow + (size_t)c * p.nN, &ldsV};
    sinkInit(su);
    sinkInit(sv);
    __syncthreads();
    const int* vprev = p.vlist + (size_t)pc * p.nN;
    const int2* vrprev = p.vlistRow + (size_t)pc * p.nN;
    const int* uprev = p.ulist + (size_t)pc * p.nN;
    const int2* rprev = p.ulistRow + (size_t)pc * p.nN;
    const unsigned stamp = (unsigned)p.ctl->totalSteps * (unsigned)(p.maxTrials + 1) + (unsigned)k;
    const double dt = p.ctl->dt;
    bool anyUnconv = false;
    int gathered = 0, live = 0, fast = 0;
    auto update = [&](int i, int2 rowIn) {
        bool listMe = false, alive = true;
        int2 row = make_int2(0, 0);
        nodeItem<false, kGeneral>(p, k, i, dt, loadNodePre(p, i, k), listMe, row, anyUnconv, gathered, live, fast,
                                  alive, rowIn);
        sinkAppend(su, listMe, i, row);
        sinkAppend(sv, alive, i, row);
    };
    for (int t = b * kBlock + (int)threadIdx.x; t < items; t += nt) {
        if (t < vc) {
            update(vprev[t], vrprev[t]);                 // A (its entry carries the row bounds)
        } else if (t >= vc + 4 * uc) {                   // C: woken by a ghost value (claimed at the unpack)
            const int n = p.xwlist[t - vc - 4 * uc];
            bool listMe = false, alive = false;
            int2 row = make_int2(0, 0);
            nodeItem<false, kGeneral>(p, k, n, dt, loadNodePre(p, n, k), listMe, row, anyUnconv, gathered, live,
                                      fast, alive);
            sinkAppend(su, listMe, n, row);
            sinkAppend(sv, alive, n, row);
        } else {                                         // B: a frozen neighbour of a listed node
            const int s = t - vc;
            const int2 rb = rprev[s >> 2];
            (void)uprev;
            for (int e = rb.x + (s & 3); e < rb.y; e += 4) {
                const int n = p.csrOther[e];
                bool mine = false;
                if (n >= 0) {
                    const int fz = p.frz[n];
                    mine = fz != 0 && fz <= k && atomicExch(&p.nstamp[n], stamp) != stamp;
                }
                if (__any(mine)) {                       // (sinkAppend's ballots: wave-uniform)
                    bool listMe = false, alive = false;
                    int2 row = make_int2(0, 0);
                    if (mine)
                        nodeItem<false, kGeneral>(p, k, n, dt, loadNodePre(p, n, k), listMe, row, anyUnconv, gathered,
                                                  live, fast, alive);
                    sinkAppend(su, mine && listMe, n, row);
                    sinkAppend(sv, mine && alive, n, row);
                }
            }
        }
    }
    sinkFlush(su, &sBase);
    sinkFlush(sv, &sBase);
    nodePassEnd(p, k, anyUnconv, gathered, live, fast, true);
    probeMark(p, k, PR_N_OUT);
}

// After k_sparse: the frozen junctions take their depth at the step's last
// iteration (what finalizeFrozen and the last k_node(k) do in the unrolled
// graph), from the iteration count the convergence flags give
__global__ __launch_bounds__(kBlock) void k_unfreeze(Params p)
{
    if (!p.freeze) return;
    bool converged;
    const int m = stepIterations(p, &converged) - 1;
    if (m <= 1) return;                               // nothing advances (finalizeFrozen)
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < p.nN; i += gridDim.x * kBlock) {
        const int fz = p.frz[i];
        if (fz) {
            p.nNewDepth[i] = frozenDepth(p, i, fz, m);
            p.frz[i] = 0;
        }
    }
}

// Init: the critical flows qCritical(i yFull / 25) (xsect.c:1612-1630) of the
// outfall conduits' enumeration depths (getYcritEnum xsect.c:1634-1696), i =
// 0..25: they depend on the section only, so the outfall prologue reads them
// instead of evaluating 26 section relations per iteration
__global__ __launch_bounds__(kBlock) void k_outfall_qcs(Params p, double* out)
{
    __shared__ double ct[5 * SWX_CIRC_N];
    stageTables(ct, p.gTables);
    for (int t = blockIdx.x * kBlock + threadIdx.x; t < 26 * p.nOutLinks; t += gridDim.x * kBlock) {
        const int j = p.outLinks[t / 26], i = t % 26;
        const uint32_t f = p.lflags[j];
        double v = 0.0;
        if (!(f & LF_NC)) {
            Geom x = loadGeom(p, j, f);
            v = qCritical<true>(x, i * (x.yFull / 25.), 0.0, ct);
        }
        out[t] = v;
    }
}

// Multi-GPU neighbour exchange (partition.h).  k_xpack: the owned links
// other ranks hold as ghosts, {newFlow, surfArea1, surfArea2, dqdh (, evap,
// seep)} each, into the send buffer (neighbour-major, the receiver's ghost
// order); k_xunpack: the received values into this rank's ghost slots.  The
// node update then sums every held node over all its links in global link
// order, exactly as on one GPU.  An iteration after convergence moves nothing.
// a received ghost value replaces the slot's previous one: when any of its
// bits changed at iteration k >= 2, the ghost link's held ends are stale
// (their sums must be gathered again: dirty, as the walk marks the ends of the
// conduits it updates), and a frozen end is woken -- claimed with k_node_list's
// stamp (so its frozen-neighbour pass does not take it twice) and listed for
// that launch (the list graphs; the unrolled k_node scans every node and
// wakes a frozen one by its dirty mark)
__device__ __forceinline__ bool ghostChanged(double oldV, double newV)
{
    return __double_as_longlong(oldV) != __double_as_longlong(newV);
}
__device__ void ghostWake(const Params& p, int l, int k)
{
    const int2 nn = p.lnodes[l];
    const unsigned stamp = (unsigned)p.ctl->totalSteps * (unsigned)(p.maxTrials + 1) + (unsigned)k;
    for (int s = 0; s < 2; s++) {
        const int n = s ? nn.y : nn.x;
        if (n < 0) continue;
        p.dirty[n] = 1;
        const int fz = p.frz[n];
        if (p.buildVlist && fz != 0 && fz <= k && atomicExch(&p.nstamp[n], stamp) != stamp)
            p.xwlist[atomicAdd(&p.xwcount[k], 1)] = n;
    }
}

__global__ __launch_bounds__(kBlock) void k_xpack(Params p, int k)
{
    if (k >= 2 && p.unconv[k - 1] == 0) return;
    for (int e = blockIdx.x * kBlock + threadIdx.x; e < p.nSend; e += gridDim.x * kBlock) {
        const int l = p.sendLink[e];
        double* o = p.xsend + (size_t)p.xF * e;
        o[0] = p.lNewFlow[l];
        o[1] = p.sa1[l];
        o[2] = p.sa2[l];
        o[3] = p.dqdh[l];
        if (p.xF > 4) {
            o[4] = p.evapLoss[l];
            o[5] = p.seepLoss[l];
        }
    }
}
__global__ __launch_bounds__(kBlock) void k_xunpack(Params p, int k)
{
    if (k >= 2 && p.unconv[k - 1] == 0) return;
    for (int g = blockIdx.x * kBlock + threadIdx.x; g < p.nGhost; g += gridDim.x * kBlock) {
        const int l = p.nL + g;
        const double* v = p.xrecv + (size_t)p.xF * g;
        if (p.xwake && k >= 2) {
            bool ch = ghostChanged(p.lNewFlow[l], v[0]) || ghostChanged(p.sa1[l], v[1]) ||
                      ghostChanged(p.sa2[l], v[2]) || ghostChanged(p.dqdh[l], v[3]);
            if (p.xF > 4) ch = ch || ghostChanged(p.evapLoss[l], v[4]) || ghostChanged(p.seepLoss[l], v[5]);
            if (ch) ghostWake(p, l, k);
        }
        p.lNewFlow[l] = v[0];
        p.sa1[l] = v[1];
        p.sa2[l] = v[2];
        p.dqdh[l] = v[3];
        if (p.xF > 4) {
            p.evapLoss[l] = v[4];
            p.seepLoss[l] = v[5];
        }
    }
}
// once per step, before the node quality: the ghost links' concentrations
// (computed by their owners in the previous step), P values each
__global__ __launch_bounds__(kBlock) void k_xpack_qual(Params p)
{
    for (int e = blockIdx.x * kBlock + threadIdx.x; e < p.nSend; e += gridDim.x * kBlock)
        for (int q = 0; q < p.P; q++)
            p.xsend[(size_t)p.P * e + q] = p.lQual[p.ctl->qualPar][(size_t)q * p.nLs + p.sendLink[e]];
}
__global__ __launch_bounds__(kBlock) void k_xunpack_qual(Params p)
{
    for (int g = blockIdx.x * kBlock + threadIdx.x; g < p.nGhost; g += gridDim.x * kBlock)
        for (int q = 0; q < p.P; q++)
            p.lQual[p.ctl->qualPar][(size_t)q * p.nLs + p.nL + g] = p.xrecv[(size_t)p.P * g + q];
}

// ---- XCHG_IPC kernels (XCtl above) -----------------------------------------
// Per Picard iteration:  k_link(k) ─ k_ipc_pack ─ k_ipc_unpack ─ k_node(k)
// ─ [k_nc] ─ k_ipc_flag.  k_ipc_pack stores this rank's sent links' values as
// granules into each neighbour's ghost area; k_ipc_unpack polls its own area
// until every ghost value of this exchange has arrived and writes the ghost
// slots; k_ipc_flag (one wave) posts the iteration's convergence flag to
// every rank and ORs the flags of all ranks into unconv[k] (dynwave.c:241-256:
// the loop ends only when every node converged).  No host, no RCCL: two
// remote-store rounds per iteration.  Every wait is bounded (p.xTimeout);
// a rank that gives up records why (xerr, host-mapped) and sets every rank's
// abort word, so the others stop waiting too and every rank's next
// swmm_step reports the failure.
__device__ __forceinline__ unsigned long long llLoad(const unsigned long long* w)
{
    return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void llStore(unsigned long long* w, unsigned seq, unsigned payload)
{
    __hip_atomic_store(w, ((unsigned long long)seq << 32) | payload, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool xAborted(const Params& p)
{
    return llLoad(p.abortW) != 0 ||
           __hip_atomic_load(p.hostAbort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}
// the iteration's launches run (the others exit at once on every rank alike)
__device__ __forceinline__ bool iterRuns(const Params& p, int k)
{
    if (k >= 2 && p.unconv[k - 1] == 0) return false;
    return !(k < 2 && stepIsSteady(p));
}
// test hook: this rank stops posting from step stallStep on (its peers time out)
__device__ __forceinline__ bool xStalled(const Params& p)
{
    return p.stallStep >= 0 && p.ctl->totalSteps >= p.stallStep;
}
// poll one granule until it carries seq; false at the deadline or on an abort
__device__ bool llWait(const Params& p, const unsigned long long* w, unsigned seq, unsigned* payload,
                       unsigned long long t0)
{
    for (unsigned it = 0;; it++) {
        const unsigned long long v = llLoad(w);
        if ((unsigned)(v >> 32) == seq) {
            *payload = (unsigned)v;
            return true;
        }
        if ((it & 15) == 15) {
            if (xAborted(p)) return false;
            if ((long long)(wall_clock64() - t0) > p.xTimeout) return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}
// a wait gave up: the record for the host (first writer's fields may mix with
// a concurrent one's; any of them is a true failure) and every rank's abort
__device__ void xFail(const Params& p, int kind, int peer, unsigned seq)
{
    const bool byPeer = xAborted(p);
    __hip_atomic_store(&p.xerr[1], kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&p.xerr[2], peer, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&p.xerr[3], (int)seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&p.xerr[0], byPeer ? 2 : 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (!byPeer)
        for (int r = 0; r < p.xRanks; r++) llStore(p.peerAbort[r], 0u, 1u);
    __threadfence_system();
}
__device__ __forceinline__ double llDouble(unsigned lo, unsigned hi)
{
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
constexpr int kMaxXF = 6;         // values per ghost link: flow, 2 surface areas, dq/dh (+ evaporation, seepage)
// The owner's side: this rank's sent links' values, as granules, into each
// receiving rank's ghost area (threads tid, tid + nthr, ... of the sends)
template <bool kQual>
__device__ void ipcPack(const Params& p, int tid, int nthr)
{
    const unsigned seq = (kQual ? p.xctl->qualSeq : p.xctl->ghostSeq) + 1;
    const int par = seq & 1, F = kQual ? p.P : p.xF;
    const double* lq = kQual ? p.lQual[p.ctl->qualPar] : nullptr;
    for (int e = tid; e < p.nSend; e += nthr) {
        const int l = p.sendLink[e];
        const XPeer X = p.xpeer[p.sendNbr[e]];
        const int gi = p.sendGi[e];
        const size_t nG = (size_t)X.nGhost;
        unsigned long long* b = (kQual ? X.qual : X.ghost) + (size_t)par * 2 * F * nG + gi;
        for (int f = 0; f < F; f++) {
            double v;
            if (kQual) v = lq[(size_t)f * p.nLs + l];
            else v = f == 0 ? p.lNewFlow[l] : f == 1 ? p.sa1[l] : f == 2 ? p.sa2[l] : f == 3 ? p.dqdh[l]
                   : f == 4 ? p.evapLoss[l] : p.seepLoss[l];
            const unsigned long long bits = (unsigned long long)__double_as_longlong(v);
            llStore(b + (size_t)(2 * f) * nG, seq, (unsigned)bits);
            llStore(b + (size_t)(2 * f + 1) * nG, seq, (unsigned)(bits >> 32));
        }
    }
}
// The receiver's side: wait for every ghost value of this exchange in this
// rank's own area and write the ghost slots (iteration k >= 2: wake the held
// ends of a ghost whose value changed).  false when a wait gave up.
template <bool kQual>
__device__ bool ipcUnpack(const Params& p, int k, int tid, int nthr)
{
    const unsigned seq = (kQual ? p.xctl->qualSeq : p.xctl->ghostSeq) + 1;
    const int par = seq & 1, F = kQual ? p.P : p.xF;
    const size_t nG = (size_t)p.nGhost;
    const unsigned long long t0 = wall_clock64();
    const unsigned long long* b = (kQual ? p.qualRx : p.ghostRx) + (size_t)par * 2 * F * nG;
    double* lq = kQual ? p.lQual[p.ctl->qualPar] : nullptr;
    for (int g = tid; g < p.nGhost; g += nthr) {
        const int l = p.nL + g;
        bool ch = false;
        // value f of the ghost from its two granules (a, c: as loaded; a
        // granule that has not arrived yet is polled); false at a give-up
        auto take = [&](int f, unsigned long long a, unsigned long long c) -> bool {
            unsigned lo = (unsigned)a, hi = (unsigned)c;
            if (((unsigned)(a >> 32) != seq && !llWait(p, b + (size_t)(2 * f) * nG + g, seq, &lo, t0)) ||
                ((unsigned)(c >> 32) != seq && !llWait(p, b + (size_t)(2 * f + 1) * nG + g, seq, &hi, t0))) {
                xFail(p, kQual ? XK_QUAL : XK_GHOST, p.ghostFrom[g], seq);
                return false;
            }
            const double v = llDouble(lo, hi);
            if (!kQual && p.xwake && k >= 2) {
                const double o = f == 0 ? p.lNewFlow[l] : f == 1 ? p.sa1[l] : f == 2 ? p.sa2[l] : f == 3 ? p.dqdh[l]
                               : f == 4 ? p.evapLoss[l] : p.seepLoss[l];
                ch = ch || ghostChanged(o, v);
            }
            if (kQual) lq[(size_t)f * p.nLs + l] = v;
            else if (f == 0) p.lNewFlow[l] = v;
            else if (f == 1) p.sa1[l] = v;
            else if (f == 2) p.sa2[l] = v;
            else if (f == 3) p.dqdh[l] = v;
            else if (f == 4) p.evapLoss[l] = v;
            else p.seepLoss[l] = v;
            return true;
        };
        // the first kMaxXF values' granules in flight at once (independent
        // uncached loads), so a ghost costs one memory round trip, not 2F
        unsigned long long w[2 * kMaxXF];
#pragma unroll
        for (int q = 0; q < 2 * kMaxXF; q++) w[q] = q < 2 * F ? llLoad(b + (size_t)q * nG + g) : 0ull;
#pragma unroll
        for (int f = 0; f < kMaxXF; f++)
            if (f < F && !take(f, w[2 * f], w[2 * f + 1])) return false;
        for (int f = kMaxXF; f < F; f++)                 // more pollutants than that
            if (!take(f, llLoad(b + (size_t)(2 * f) * nG + g), llLoad(b + (size_t)(2 * f + 1) * nG + g)))
                return false;
        if (ch) ghostWake(p, l, k);
    }
    return true;
}
template <bool kQual>
__global__ __launch_bounds__(kBlock) void k_ipc_pack(Params p, int k)
{
    if (!kQual && !iterRuns(p, k)) return;
    if (xAborted(p) || xStalled(p)) return;
    ipcPack<kQual>(p, blockIdx.x * kBlock + threadIdx.x, gridDim.x * kBlock);
}
template <bool kQual>
__global__ __launch_bounds__(kBlock) void k_ipc_unpack(Params p, int k)
{
    if (!kQual && !iterRuns(p, k)) return;
    if (xAborted(p)) return;
    (void)ipcUnpack<kQual>(p, k, blockIdx.x * kBlock + threadIdx.x, gridDim.x * kBlock);
}
// Pack and unpack in one launch (one kernel boundary less per exchange:
// tools/ipc_signal_probe measures 3.0-3.3 against 4.1-4.4 us per iteration;
// opt-in, SWMM5_XCHG_FUSED=1).
// Every workgroup posts its share of the sends before it waits for anything,
// and the grid (kXchgGrid workgroups) is small enough to be resident at once,
// so every rank's posts are made whatever its waiting workgroups hold.
constexpr int kXchgGrid = 128;
template <bool kQual>
__global__ __launch_bounds__(kBlock) void k_ipc_xchg(Params p, int k)
{
    if (!kQual && !iterRuns(p, k)) return;
    if (xAborted(p)) return;
    const int tid = blockIdx.x * kBlock + threadIdx.x, nthr = gridDim.x * kBlock;
    if (!xStalled(p)) ipcPack<kQual>(p, tid, nthr);
    (void)ipcUnpack<kQual>(p, k, tid, nthr);
}
// One wave: iteration k's flag from every rank, ORed into unconv[k] (the
// all-reduce(max) of the RCCL transport); kHello: the start-up handshake
// (flag exchange number 1 with every rank's flag 1; *out = 1 when it worked)
template <bool kHello>
__global__ __launch_bounds__(64) void k_ipc_flag(Params p, int k, int* out)
{
    if (!kHello && !iterRuns(p, k)) return;
    const int t = threadIdx.x;
    const unsigned seq = p.xctl->flagSeq + 1;
    const int par = seq & 1, R = p.xRanks;
    bool ok = !xAborted(p);
    if (ok && t < R && !(!kHello && xStalled(p))) {
        const unsigned mine = kHello ? 1u : (p.unconv[k] != 0 ? 1u : 0u);
        llStore(p.peerFlag[t] + (size_t)par * R + p.xRank, seq, mine);
    }
    unsigned v = 0;
    const unsigned long long t0 = wall_clock64();
    if (ok && t < R) ok = llWait(p, p.flagRx + (size_t)par * R + t, seq, &v, t0);
    const unsigned long long m = __ballot(!ok && t < R);
    const bool any = __any(ok && t < R && v != 0);
    if (m) {                                       // the lowest failing lane records it
        if (t == __ffsll((long long)m) - 1) xFail(p, kHello ? XK_HELLO : XK_FLAG, t, seq);
        if (kHello && t == 0) *out = 0;
        return;
    }
    if (t == 0) {
        if (kHello) *out = any ? 1 : 0;
        else p.unconv[k] = any ? 1 : 0;
        p.xctl->flagSeq = seq;
        if (!kHello) p.xctl->ghostSeq += 1;        // this iteration's ghost exchange is complete
    }
}
// One wave: n <= kRedMax doubles reduced over the ranks in rank order (op 0
// sum, 1 min), in place -- the same value on every rank
__global__ __launch_bounds__(64) void k_ipc_reduce(Params p, double* vals, int n, int op)
{
    __shared__ double sv[64][kRedMax];
    __shared__ int okAll;
    const int t = threadIdx.x;
    const unsigned seq = p.xctl->redSeq + 1;
    const int par = seq & 1, R = p.xRanks;
    const size_t slot = 2 * kRedMax;
    bool ok = !xAborted(p);
    if (ok && t < R && !xStalled(p)) {
        unsigned long long* w = p.peerRed[t] + ((size_t)par * R + p.xRank) * slot;
        for (int i = 0; i < n; i++) {
            const unsigned long long bits = (unsigned long long)__double_as_longlong(vals[i]);
            llStore(w + 2 * i, seq, (unsigned)bits);
            llStore(w + 2 * i + 1, seq, (unsigned)(bits >> 32));
        }
    }
    const unsigned long long t0 = wall_clock64();
    if (ok && t < R) {
        const unsigned long long* w = p.redRx + ((size_t)par * R + t) * slot;
        for (int i = 0; i < n && ok; i++) {
            unsigned lo = 0, hi = 0;
            ok = llWait(p, w + 2 * i, seq, &lo, t0) && llWait(p, w + 2 * i + 1, seq, &hi, t0);
            sv[t][i] = llDouble(lo, hi);
        }
    }
    const unsigned long long m = __ballot(!ok && t < R);
    if (t == 0) okAll = m == 0;
    __syncthreads();
    if (!okAll) {
        if (m && t == __ffsll((long long)m) - 1) xFail(p, XK_RED, t, seq);
        return;
    }
    if (t == 0) {
        for (int i = 0; i < n; i++) {
            double a = sv[0][i];
            for (int r = 1; r < R; r++) a = op ? (sv[r][i] < a ? sv[r][i] : a) : a + sv[r][i];
            vals[i] = a;
        }
        p.xctl->redSeq = seq;
    }
}

// ---------------------------------------------------------------------------
// Non-conduit links (findLinkFlows' second loop, dynwave.c:404-412, and
// findNonConduitFlow / getModPumpFlow / findNonConduitSurfArea /
// updateNodeFlows, dynwave.c:423-590), then the depths of their end nodes
// (setNodeDepth).  One workgroup: the flow of every regulator depends only on
// last iteration's depths and runs in parallel; a pump's inlet limits and the
// node sums need the running node totals in link order, which one thread
// accumulates; the deferred nodes then update in parallel.
__device__ __forceinline__ double ncDepth(const Params& p, int n)
{
    // an outfall's depth was refreshed by this iteration's k_node prologue;
    // the link flows of the reference use the previous one
    return ((int)(p.nflags[n] & NF_TYPE) == OUTFALL) ? p.nPrevDepth[n] : p.nNewDepth[n];
}

template <bool kFirst>
__global__ __launch_bounds__(kBlock) void k_nc(Params p, int k)
{
    if (k >= 2 && p.unconv[k - 1] == 0) return;
    if (k < 2 && stepIsSteady(p)) return;            // SKIP_STEADY_STATE
    __shared__ double ct[5 * SWX_CIRC_N];
    __shared__ int anyU;
    stageTables(ct, p.gTables);
    if (threadIdx.x == 0) anyU = 0;
    const double dt = p.ctl->dt;
    const double ucfV = p.ucfV;
    if (kFirst) {
        // link_setOldHydState + link_setTargetSetting / link_setSetting for
        // pumps (routing.c:214-227, link.c:604-640), node_initFlows overflow
        for (int c = threadIdx.x; c < p.nNC; c += kBlock) {
            int j = p.ncLinks[c];
            p.lOldFlow[j] = p.lNewFlow[j];
            p.lOldDepth[j] = p.lNewDepth[j];
            p.lOldVolume[j] = p.lNewVolume[j];
            const NcLink& L = p.ncL[c];
            double set = p.setting[j], ts = p.ncTarget[c];
            if (L.type == LK_PUMP) {
                int n1 = p.lnodes[j].x;
                double y1 = p.nOldDepth[n1];
                ts = set;
                if (L.yOff > 0.0 && set > 0.0 && y1 < L.yOff) ts = 0.0;
                if (L.yOn > 0.0 && set == 0.0 && y1 > L.yOn) ts = 1.0;
                if (ts != set) p.setting[j] = ts;
            }
            p.ncTarget[c] = ts;
        }
        for (int d = threadIdx.x; d < p.nDef; d += kBlock) {
            int i = p.defNodes[d];
            if ((int)(p.nflags[i] & NF_TYPE) == OUTFALL) continue;
            double v = p.nNewVolume[i], fv = p.fullVolume[i];
            p.overflow[i] = (v > fv) ? (v - fv) / dt : 0.0;
        }
        __syncthreads();
    }
    // ---- phase A: regulator / pump-curve flows from last iteration's depths
    for (int c = threadIdx.x; c < p.nNC; c += kBlock) {
        int j = p.ncLinks[c];
        int2 nn = p.lnodes[j];
        int byp = (k >= 2 && p.conv[nn.x] && p.conv[nn.y]) ? 1 : 0;   // findBypassedLinks
        p.ncBypass[c] = byp;
        if (byp) continue;
        const NcLink& L = p.ncL[c];
        uint32_t f = p.lflags[j];
        double qLast = p.lNewFlow[j];
        NcOut o;
        o.dqdh = 0.0;
        o.depth = p.lNewDepth[j];
        o.surfArea = p.ncSurf[c];
        o.flowClass = p.lstate[j] & 0xF;
        double set = p.setting[j], q = 0.0;
        double y1 = ncDepth(p, nn.x), y2 = ncDepth(p, nn.y);
        double inv1 = p.invert[nn.x], inv2 = p.invert[nn.y];
        bool of1 = (f & LF_N1_OFLAP) != 0, of2 = (f & LF_N2_OFLAP) != 0;
        const double* cx = p.curveX + L.cOff;
        const double* cy = p.curveY + L.cOff;
        NcCoef cf;
        cf.cOrif = p.ncCoef[4 * c];
        cf.cWeir = p.ncCoef[4 * c + 1];
        cf.hCrit = p.ncCoef[4 * c + 2];
        cf.cSurcharge = p.ncCoef[4 * c + 3];
        if (set != 0.0) {                                   // link_getInflow (link.c:543-560)
            Geom g = loadGeom<false>(p, j, f);
            switch (L.type) {
            case LK_ORIFICE: q = orificeInflow(L, g, cf, set, y1, y2, inv1, inv2, of1, of2, &o, ct); break;
            case LK_WEIR: q = weirInflow(L, g, cf, cx, cy, set, y1, y2, inv1, inv2, of1, of2, &o, ct); break;
            case LK_OUTLET: q = outletInflow(L, cx, cy, set, y1, y2, inv1, inv2, of1, of2, &o); break;
            case LK_PUMP:
                set = p.ncTarget[c];                        // pump_getInflow (link.c:1564-1566)
                p.setting[j] = set;
                o.flowClass = 0;
                if (set != 0.0 && L.sub != PT_IDEAL)
                    q = pumpInflow(L, cx, cy, set, y1, y2, inv1, inv2, p.nNewVolume[nn.x], ucfV, &o);
                break;
            }
        }
        // findNonConduitSurfArea (dynwave.c:510-525)
        double sa1 = (L.type == LK_ORIFICE) ? o.surfArea / 2. : 0.0, sa2 = sa1;
        if (L.type == LK_ORIFICE || L.type == LK_WEIR) p.ncSurf[c] = o.surfArea;
        if (o.flowClass == FC_UP_CRITICAL || (int)(p.nflags[nn.x] & NF_TYPE) == STORAGE) sa1 = 0.0;
        if (o.flowClass == FC_DN_CRITICAL || (int)(p.nflags[nn.y] & NF_TYPE) == STORAGE) sa2 = 0.0;
        p.sa1[j] = sa1;
        p.sa2[j] = sa2;
        p.dqdh[j] = o.dqdh;
        p.lNewDepth[j] = o.depth;
        p.lstate[j] = (p.lstate[j] & ~0xF) | (o.flowClass & 0xF);
        if (L.type == LK_PUMP) {
            p.ncQ[c] = q;
        } else if (L.type == LK_CONDUIT) {
            // DUMMY conduit: its flow is its upstream node's outflow at its
            // turn in link order (phase B)
        } else {
            if (k > 0) {                                    // under-relaxation (dynwave.c:455-461)
                q = (1.0 - 0.5) * qLast + 0.5 * q;
                if (q * qLast < 0.0) q = 0.001 * ((q < 0.0) ? -1.0 : 1.0);
            }
            p.lNewFlow[j] = q;
        }
    }
    __syncthreads();
    // ---- phase B: link-order accumulation into the end nodes (one thread)
    if (threadIdx.x == 0) {
        for (int c = 0; c < p.nNC; c++) {
            int j = p.ncLinks[c];
            int2 nn = p.lnodes[j];
            const NcLink& L = p.ncL[c];
            int n1 = nn.x, n2 = nn.y;
            if (L.type == LK_PUMP && !p.ncBypass[c]) {
                double q = p.ncQ[c];
                double set = p.setting[j];
                if (L.sub == PT_IDEAL && set != 0.0) {      // pump_getInflow IDEAL_PUMP
                    q = p.inflow[n1] + p.overflow[n1];
                    if (q < 0.0) q = 0.0;
                    q = q * set;
                }
                if (q != 0.0) {                             // getModPumpFlow (dynwave.c:466-503)
                    bool maxOut = (int)(p.nflags[n1] & NF_TYPE) == STORAGE || L.sub == PT_TYPE1;
                    if (maxOut) {                           // node_getMaxOutflow (node.c:418-434)
                        if (p.fullVolume[n1] > 0.0) {
                            double qMax = p.inflow[n1] + p.nOldVolume[n1] / dt;
                            if (q > qMax) q = qMax;
                        }
                        q = gmax(0.0, q);
                    } else if (L.sub == PT_TYPE2 || L.sub == PT_TYPE3 || L.sub == PT_TYPE4) {
                        double newNet = p.inflow[n1] - p.outflow[n1] - q;
                        double vol = 0.5 * (p.oldNetInflow[n1] + newNet) * dt;
                        double y = p.nOldDepth[n1] + vol / p.nSurf[n1];
                        if (y <= 0.0) q = p.inflow[n1];
                    }
                }
                p.lNewFlow[j] = q;
            } else if (L.type == LK_CONDUIT && !p.ncBypass[c]) {
                // DUMMY conduit (findNonConduitFlow dynwave.c:423-461):
                // link_getInflow -> conduit_getInflow (link.c:543-560,
                // 1320-1330) = node_getOutflow of its upstream node (a junction:
                // inflow + overflow so far, node.c:400-414), capped by its flow
                // limit, then under-relaxed (not a pump)
                const double qLast = p.lNewFlow[j];
                double q = 0.0;
                if (p.setting[j] != 0.0) {
                    q = p.inflow[n1] + p.overflow[n1];
                    if (L.qLimit > 0.0) q = gmin(q, L.qLimit);
                }
                if (k > 0) {
                    q = (1.0 - 0.5) * qLast + 0.5 * q;
                    if (q * qLast < 0.0) q = 0.001 * ((q < 0.0) ? -1.0 : 1.0);
                }
                p.lNewFlow[j] = q;
            }
            // updateNodeFlows (dynwave.c:531-590)
            double q = p.lNewFlow[j];
            if (q >= 0.0) { p.outflow[n1] += q; p.inflow[n2] += q; }
            else { p.inflow[n1] -= q; p.outflow[n2] -= q; }
            p.nSurf[n1] += p.sa1[j];
            p.nSurf[n2] += p.sa2[j];
            double dq = p.dqdh[j];
            p.nDqdh[n1] += dq;
            if (!(L.type == LK_PUMP && L.sub == PT_TYPE4)) p.nDqdh[n2] += dq;
        }
        __threadfence();
    }
    __syncthreads();
    // ---- phase C: setNodeDepth for the deferred nodes
    bool anyUnconv = false;
    int* ulist = p.ulist + (size_t)(k & 1) * p.nN;
    int2* urow = p.ulistRow + (size_t)(k & 1) * p.nN;
    for (int base = 0; base < p.nDef; base += kBlock) {
        int d = base + threadIdx.x;
        bool listMe = false;
        int2 row = make_int2(0, 0);
        if (d < p.nDef) {
            int i = p.defNodes[d];
            row = make_int2(p.rowptr[i], p.rowptr[i + 1]);
            uint32_t nf = p.nflags[i];
            if ((int)(nf & NF_TYPE) != OUTFALL) {
                double yLast = p.nNewDepth[i], yOld = p.nOldDepth[i];
                if (!(nodeUpdate(p, i, k, nf, dt, yLast, yOld, p.inflow[i], p.outflow[i], p.nSurf[i],
                                 p.nDqdh[i]) & 1)) {
                    anyUnconv = true;
                    listMe = true;
                }
            }
        }
        if (!kFirst) waveAppend(listMe, d < p.nDef ? p.defNodes[d] : -1, row, &p.ucount[k], ulist, urow);
    }
    if (anyUnconv) anyU = 1;
    __syncthreads();
    if (threadIdx.x == 0 && anyU) p.unconv[k] = 1;
}

// qualrout.c:146-174, 498-518
__device__ __forceinline__ double mixedQual(double c, double v1, double wIn, double qIn, double tStep)
{
    if (qIn <= 1.E-10) return c;
    double vIn = qIn * tStep;
    double cIn = wIn * tStep / vIn;
    double cMax = gmax(c, cIn);
    c = (c * v1 + wIn * tStep) / (v1 + vIn);
    c = gmin(c, cMax);
    c = gmax(c, 0.0);
    return c;
}
__device__ __forceinline__ double reactedQual(double kDecay, double c, double tStep)
{
    if (kDecay == 0.0) return c;
    double c2 = c * (1.0 - kDecay * tStep);
    return gmax(0.0, c2);
}

// qualrout.c:100-142 in one pass over the nodes: each node's mass inflow
// from its downstream-flowing links (findLinkMassFlow, link order), its new
// quality (findNodeQual / findStorageQual), then the quality of every link
// the node feeds (findLinkQual: a link's quality needs only its upstream
// node's new quality and its own state, so the thread that has just computed
// that node updates it; each link has exactly one upstream end).  Old values
// are read from buffer [qualPar], new ones written to [qualPar ^ 1], so no
// thread reads a concentration another one writes.
// One node of qualrout_execute (the body of k_qual_node's loop; k_step_end
// runs it too, fused, for networks with pollutants: kQual)
__device__ __forceinline__ void qualNode(const Params& p, int i, double dt, const double* nOld, double* nNew,
                                         const double* lOld, double* lNew)
{
    const double depth = p.nNewDepth[i];
    double qIn = p.inflow[i];
    double oldVol = p.nOldVolume[i];
    int e0 = p.qrowptr[i], e1 = p.qrowptr[i + 1];
    const bool isStorage = (int)(p.nflags[i] & NF_TYPE) == STORAGE;
    double fEvap = 1.0;
    if (isStorage) {                     // findStorageQual (qualrout.c:417-436)
        double h = p.hrt[i];             // updateHRT (qualrout.c:478-494)
        if (oldVol < 1.E-10) h = 0.0;
        else h = (h + dt) * oldVol / (oldVol + qIn * dt);
        p.hrt[i] = gmax(h, 0.0);
        double vEvap = p.nEvapVol[i];
        if (vEvap > 0.0 && oldVol > 0.0353147) fEvap += vEvap / oldVol;
    }
    // mass inflow of every pollutant in one pass over the node's links
    // (each pollutant's sum in link order, as qualrout.c:162-174 adds it)
    double wq[kQualBatch], cn[kQualBatch];
    for (int p0 = 0; p0 < p.P; p0 += kQualBatch) {
    const int np = (p.P - p0 < kQualBatch) ? p.P - p0 : kQualBatch;
    for (int b = 0; b < np; b++) wq[b] = p.qualIn[(size_t)(p0 + b) * p.nN + i];
    // kQGather CSR entries at a time: their words, then their flows, then
    // the downstream-flowing links' concentrations load together before
    // the in-order sums (one entry at a time is three dependent loads each)
    for (int eb = e0; eb < e1; eb += kQGather) {
        int ent[kQGather];
        double ql[kQGather], lo[kQGather][kQualBatch];
        bool down[kQGather];
#pragma unroll
        for (int t = 0; t < kQGather; t++) ent[t] = (eb + t < e1) ? p.qcsr[eb + t] : 0;
#pragma unroll
        for (int t = 0; t < kQGather; t++) ql[t] = (eb + t < e1) ? p.lNewFlow[ent[t] & 0x7FFFFFFF] : 0.0;
#pragma unroll
        for (int t = 0; t < kQGather; t++) {
            down[t] = (eb + t < e1) && ((ent[t] < 0) ? !(ql[t] < 0.0) : (ql[t] < 0.0));
#pragma unroll
            for (int b = 0; b < kQualBatch; b++)
                lo[t][b] = (down[t] && b < np) ? lOld[(size_t)(p0 + b) * p.nLs + (ent[t] & 0x7FFFFFFF)] : 0.0;
        }
#pragma unroll
        for (int t = 0; t < kQGather; t++) {
            if (!down[t]) continue;
            const double aq = fabs(ql[t]);
#pragma unroll
            for (int b = 0; b < kQualBatch; b++)
                if (b < np) wq[b] += aq * lo[t][b];
        }
    }
    for (int b = 0; b < np; b++) {
        const int pp = p0 + b;
        size_t ni = (size_t)pp * p.nN + i;
        double cOld = nOld[ni];                 // node_setOldQualState: old <- new (buffer flip)
        double w = wq[b];
        double c;
        if (isStorage || oldVol > 0.0353147) {
            double c1 = reactedQual(p.kDecay[pp], cOld * fEvap, dt);
            c = mixedQual(c1, oldVol, w, qIn, dt);
            if ((p.nNewVolume[i] <= 0.0353147 || depth <= 0.003281) && qIn <= 1.E-10) c = 0.0;
        } else if (qIn > 1.E-10) {
            c = w / qIn;
        } else {
            c = (depth > 0.003281) ? cOld : 0.0;
        }
        nNew[ni] = c;
        cn[b] = c;
    }
    // findLinkQual (qualrout.c:253-353, DW) of the links this node feeds,
    // kQGather CSR entries at a time (their state loads together)
    for (int eb = e0; eb < e1; eb += kQGather) {
        int ent[kQGather];
        double ql[kQGather];
#pragma unroll
        for (int t = 0; t < kQGather; t++) ent[t] = (eb + t < e1) ? p.qcsr[eb + t] : 0;
#pragma unroll
        for (int t = 0; t < kQGather; t++) ql[t] = (eb + t < e1) ? p.lNewFlow[ent[t] & 0x7FFFFFFF] : 0.0;
        bool up[kQGather];
        uint32_t fl[kQGather];
        double q1v[kQGather], sl[kQGather], el[kQGather], v1v[kQGather], v2v[kQGather], dl[kQGather];
        double lo[kQGather][kQualBatch];
#pragma unroll
        for (int t = 0; t < kQGather; t++) {
            const int l = ent[t] & 0x7FFFFFFF;
            // a ghost link (l >= nL): its owner updates it
            up[t] = (eb + t < e1) && l < p.nL && ((ent[t] < 0) ? (ql[t] < 0.0) : !(ql[t] < 0.0));
            fl[t] = up[t] ? p.lflags[l] : 0u;
            q1v[t] = up[t] ? p.q1[l] : 0.0;
            // (0 for a link without LF_SEEP, never rewritten: not loaded
            // when no held link has losses, p.xF == 4)
            sl[t] = (up[t] && p.xF > 4) ? p.seepLoss[l] : 0.0;
            el[t] = (up[t] && p.xF > 4) ? p.evapLoss[l] : 0.0;
            v1v[t] = up[t] ? p.lOldVolume[l] : 0.0;
            v2v[t] = up[t] ? p.lNewVolume[l] : 0.0;
            dl[t] = up[t] ? p.lNewDepth[l] : 0.0;
#pragma unroll
            for (int b = 0; b < kQualBatch; b++)
                lo[t][b] = (up[t] && b < np) ? lOld[(size_t)(p0 + b) * p.nLs + l] : 0.0;
        }
#pragma unroll
        for (int t = 0; t < kQGather; t++) {
            if (!up[t]) continue;
            const int l = ent[t] & 0x7FFFFFFF;
            const uint32_t f = fl[t];
            if (f & LF_NC) {                    // non-conduit: its upstream node's quality (qualrout.c:283-291)
#pragma unroll
                for (int b = 0; b < kQualBatch; b++)
                    if (b < np) lNew[(size_t)(p0 + b) * p.nLs + l] = cn[b];
                continue;
            }
            double barrels = (double)((f >> LF_BARREL_SHIFT) & 0xFF);
            double lq = fabs(q1v[t]) * barrels;
            double qSeep = sl[t] * barrels;
            double vEvap = el[t] * barrels * dt;
            double v1 = v1v[t], v2 = v2v[t];
            double vLosses = qSeep * dt + vEvap;
            double fe = 1.0;
            if (vEvap > 0.0 && v1 > 0.0353147) fe += vEvap / v1;
            lq = lq + (v2 + vLosses - v1) / dt;
            lq = gmax(lq, 0.0);
            bool dry = (v2 < 0.0353147 || dl[t] <= 0.003281);
#pragma unroll
            for (int b = 0; b < kQualBatch; b++) {
                if (b >= np) continue;
                const int pp = p0 + b;
                size_t li = (size_t)pp * p.nLs + l;
                double c1 = lo[t][b] * fe;
                double c2 = reactedQual(p.kDecay[pp], c1, dt);
                double wIn = cn[b] * lq;
                c2 = mixedQual(c2, v1, wIn, lq, dt);
                if (dry) c2 = 0.0;
                lNew[li] = c2;
            }
        }
    }
    }
}

// (four waves per SIMD -- 128 VGPRs, 52 B of spills -- measured 63.9-64.4
// against 61.3 us on the 1M P = 3 grid: three it is)
__global__ __launch_bounds__(kBlock) void k_qual_node(Params p)
{
    const double dt = p.ctl->dt;
    const int par = p.ctl->qualPar;
    const double* nOld = p.nQual[par];
    double* nNew = p.nQual[par ^ 1];
    const double* lOld = p.lQual[par];
    double* lNew = p.lQual[par ^ 1];
    int m = 0;
    if (p.qualUnfreeze) {
        bool converged;
        m = stepIterations(p, &converged) - 1;
    }
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < p.nN; i += gridDim.x * kBlock) {
        if (p.qualUnfreeze) {                         // k_unfreeze's work for this node (qualNode reads only
            const int fz = p.frz[i];                  // its own node's depth)
            if (fz) {
                p.nNewDepth[i] = frozenDepth(p, i, fz, m);
                p.frz[i] = 0;
            }
        }
        qualNode(p, i, dt, nOld, nNew, lOld, lNew);
    }
}

// getVariableStep (dynwave.c:799-832) from the uncapped link and node
// Courant minima: getLinkStep(maxStep) then getNodeStep(tMinLink), the
// absolute minimum, then the millisecond floor of dynwave_getRoutingStep.
// *crit: 2 = a node, 1 = a link set the step (stats_updateCriticalTimeCount),
// 0 = the cap did
__host__ __device__ inline double courantStep(double linkMin, double nodeMin, double maxStep,
                                              double minStep, int* crit)
{
    double tMinLink = maxStep;
    *crit = 0;
    if (linkMin < tMinLink) { tMinLink = linkMin; *crit = 1; }
    double tMin = tMinLink;
    if (nodeMin < tMinLink) { tMin = nodeMin; *crit = 2; }
    if (tMin < minStep) tMin = minStep;
    return floor(1000.0 * tMin) / 1000.0;
}

// combine two partial vectors (sums; mins keep the first occurrence)
__device__ __forceinline__ void combinePartials(double* a, const double* b)
{
    for (int q = 0; q < kNumPartials; q++) {
        if (q == 8 || q == 9) continue;
        if (partialIsMin(q)) {
            if (b[q] < a[q] || (b[q] == a[q] && b[q + 3] < a[q + 3])) { a[q] = b[q]; a[q + 3] = b[q + 3]; }
        } else {
            a[q] += b[q];
        }
    }
}

// link_getVelocity (link.c:809-830) for a conduit
template <bool kFast, bool kAll>
__device__ __forceinline__ double conduitVelocity(const Params& p, int j, uint32_t f, double q, double depth,
                                                  const double* ct)
{
    if (depth <= 0.01) return 0.0;
    double barrels = (double)((f >> LF_BARREL_SHIFT) & 0xFF);
    q /= barrels;
    Geom x = loadGeom<kFast>(p, j, f, ct);
    double area = getAofY<kAll>(x, depth, ct);
    return (area > 0.0001) ? q / area : 0.0;
}

// Step end: findLimitedLinks (dynwave.c:349-378), removeConduitLosses /
// removeOutflows (routing.c:841-925, node.c:438-493), Courant partials
// (dynwave.c:836-921), run statistics (stats_updateFlowStats, stats.c:449-752)
// and the per-node volume totals (massbal_updateRoutingTotals, massbal.c:619-633).
// Block partials: see kNumPartials.
// kQual: qualrout_execute fused into the node pass (qualNode before the
// node's step-end work; every value it reads is the node's own or a link's,
// and no step-end write touches them), one launch and one read of the
// shared node state instead of two
template <bool kFast, bool kAll, bool kQual = false>
__global__ __launch_bounds__(kBlock) void k_step_end(Params p)
{
    __shared__ double red[kNumPartials][kBlock / 64];
    __shared__ double ct[kFast ? kCtFast : 5 * SWX_CIRC_N];
    stageTables(ct, p.gTables, kFast ? p.nGeom : 0);
    double acc[kNumPartials];
    for (int q = 0; q < kNumPartials; q++) acc[q] = 0.0;
    // Courant limits uncapped: k_finalize caps them with the routing step in
    // force when the next step begins (swmm_stride may lower it meanwhile)
    acc[5] = 1.0e300; acc[8] = 1.0e300;
    acc[6] = 1.0e300; acc[9] = 1.0e300;
    StepCtl* c = p.ctl;
    const double dt = c->dt;
    const double half = dt / 2.;
    // date at the end of this step (getDateTime(NewRoutingTime), swmm5.c:1543)
    const double tEnd = c->newRoutingTime + 1000.0 * c->dt;
    const double aDate = c->dateBase + (c->dateSecs0 + (tEnd + 1) / 1000.0) / 86400.0;
    const bool stats = !(aDate < c->statsStart);
    // convergence of this step (dynwave.c:242-257): nodes count non-convergence
    bool converged;
    [[maybe_unused]] const int steps = stepIterations(p, &converged);
    const StatsDev& S = p.st;
    // a step skipped as steady: findLimitedLinks and setNodeDepth's dYdT
    // belong to dynwave_execute, which did not run (routing.c:239-241)
    const bool steady = stepIsSteady(p);
    int n = gridDim.x * kBlock;
    int tid = blockIdx.x * kBlock + threadIdx.x;
    // the live count after iteration 1 (blockLive, k_node(1)); 0 when the
    // step converged at iteration 0 or 1 and k_node(1) wrote nothing new --
    // then the values of an earlier step, harmless for a heuristic
    for (int b = tid; b < p.blockLiveN; b += n) acc[10] += (double)p.blockLive[b];
    // links (fixed order within a thread: j = tid, tid + n, ...)
    for (int j = tid; j < p.nL; j += n) {
        uint32_t f = p.lflags[j];
        if (f & LF_NC) {                                   // stats_updateLinkStats, non-conduits
            if (!stats) continue;
            double newFlow = p.lNewFlow[j], oldFlow = p.lOldFlow[j];
            double dq = newFlow - oldFlow;
            double q = fabs(newFlow);
            if (q > S.lMaxFlow[j]) { S.lMaxFlow[j] = q; S.lMaxFlowDate[j] = aDate; }
            double depth = p.lNewDepth[j];
            if (depth > S.lMaxDepth[j]) S.lMaxDepth[j] = depth;
            if (f & LF_PUMP) {
                if (q >= S.qFull[j]) S.lTimeFullFlow[j] += dt;
                if (q > 0.001) {
                    int2 nn = p.lnodes[j];
                    p.pMin[j] = gmin(p.pMin[j], q);
                    p.pMax[j] = S.lMaxFlow[j];
                    p.pAvg[j] += q;
                    p.pVol[j] += q * dt;
                    p.pUtil[j] += dt;
                    double dh = (p.invert[nn.x] + p.nNewDepth[nn.x]) - (p.invert[nn.y] + p.nNewDepth[nn.y]);
                    double power = fabs(dh) * q / 8.814 * 0.7457;          // link_getPower
                    p.pEnergy[j] += power * dt / 3600.0;
                    int fc = p.lstate[j] & 0xF;
                    if (fc == FC_DN_DRY) p.pOffLow[j] += dt;
                    if (fc == FC_UP_DRY) p.pOffHigh[j] += dt;
                    if (oldFlow < 0.001) p.pStarts[j] += 1;
                    p.pPeriods[j] += 1;
                    S.lTimeSurch[j] += dt;
                    S.lTimeFullUp[j] += dt;
                    S.lTimeFullDn[j] += dt;
                }
            }
            if (f & LF_DUMMY) {                            // still a CONDUIT (stats.c:707-745)
                const int s = p.lstate[j];
                if (s & (1 << 8)) S.lTimeNormal[j] += dt;
                if (s & (1 << 10)) S.lTimeInlet[j] += dt;
                const int fc = s & 0xF;
                if (fc < 7) S.lTimeClass[(size_t)fc * p.nL + j] += dt;
                if (q >= S.qFull[j] * (double)((f >> LF_BARREL_SHIFT) & 0xFF)) S.lTimeFullFlow[j] += dt;
                if (s & (1 << 9)) S.lTimeCapLim[j] += dt;
                const int fs = (s >> 4) & 0xF;
                if (fs == FS_ALL_FULL) {
                    S.lTimeSurch[j] += dt;
                    S.lTimeFullUp[j] += dt;
                    S.lTimeFullDn[j] += dt;
                } else if (fs == FS_UP_FULL) {
                    S.lTimeFullUp[j] += dt;
                } else if (fs == FS_DN_FULL) {
                    S.lTimeFullDn[j] += dt;
                }
            }
            int k0 = S.lTurnSign[j];
            int sg = (dq < 0) ? -1 : 1;
            S.lTurnSign[j] = sg;
            if (fabs(dq) > 0.001 && k0 * sg < 0) S.lTurns[j] += 1;
            continue;
        }
        double barrels = (double)((f >> LF_BARREL_SHIFT) & 0xFF);
        const int skip = p.endSkip | (steady ? 64 : 0);
        int s = steady ? p.lstate[j] : (p.lstate[j] & ~(1 << 9));
        double a1 = p.a1[j];
        if (!(skip & 64) && a1 >= p.aFull[j]) {
            int2 nn = p.lnodes[j];
            double h1 = p.nNewDepth[nn.x] + p.inv1[j];
            double h2 = p.nNewDepth[nn.y] + p.inv2[j];
            if ((h1 - h2) > fabs(p.slope[j]) * p.lengthRaw[j]) s |= (1 << 9);
        }
        if (!(skip & 64)) p.lstate[j] = s;
        if (f & LF_SEEP) {
            acc[3] += p.evapLoss[j] * barrels;
            acc[4] += p.seepLoss[j] * barrels;
        }
        double newFlow = p.lNewFlow[j];
        if (p.varStep && !(skip & 32)) {
            double q = fabs(newFlow) / barrels;
            double fr = p.froude[j];
            if (!(q <= 0.0001 || a1 <= 0.0001 || fr <= 0.01)) {
                double t = p.lNewVolume[j] / barrels / q;
                t = t * p.modLength[j] / p.length[j];
                t = t * fr / (1.0 + fr) * p.courantFactor;
                if (t < acc[5]) { acc[5] = t; acc[8] = (double)j; }
            }
        }
        if (stats && !(skip & 1)) {                        // stats_updateLinkStats
            double dq = newFlow - p.lOldFlow[j];
            double q = fabs(newFlow);
            double depth = p.lNewDepth[j];
            if (!(skip & 4)) {
                if (q > S.lMaxFlow[j]) { S.lMaxFlow[j] = q; S.lMaxFlowDate[j] = aDate; }
                double v = (f & LF_COLD) ? conduitVelocity<false, kAll>(p, j, f, q, depth, ct)
                                         : conduitVelocity<kFast, false>(p, j, f, q, depth, ct);
                if (v > S.lMaxVeloc[j]) S.lMaxVeloc[j] = v;
                if (depth > S.lMaxDepth[j]) S.lMaxDepth[j] = depth;
            }
            if (s & (1 << 8)) S.lTimeNormal[j] += dt;
            if (s & (1 << 10)) S.lTimeInlet[j] += dt;
            int fc = s & 0xF;
            if (fc < 7 && !(skip & 2)) S.lTimeClass[(size_t)fc * p.nL + j] += dt;
            if (q >= S.qFull[j] * barrels) S.lTimeFullFlow[j] += dt;
            if (s & (1 << 9)) S.lTimeCapLim[j] += dt;
            int fs = (s >> 4) & 0xF;
            if (fs == FS_ALL_FULL) {
                S.lTimeSurch[j] += dt;
                S.lTimeFullUp[j] += dt;
                S.lTimeFullDn[j] += dt;
            } else if (fs == FS_UP_FULL) {
                S.lTimeFullUp[j] += dt;
            } else if (fs == FS_DN_FULL) {
                S.lTimeFullDn[j] += dt;
            }
            int k = S.lTurnSign[j];
            int sg = (dq < 0) ? -1 : 1;
            S.lTurnSign[j] = sg;
            if (fabs(dq) > 0.001 && k * sg < 0) S.lTurns[j] += 1;
        }
    }
    for (int i = tid; i < p.nN; i += n) {
        if (kQual) {
            const int par = c->qualPar;
            qualNode(p, i, dt, p.nQual[par], p.nQual[par ^ 1], p.lQual[par], p.lQual[par ^ 1]);
        }
        uint32_t nf = p.nflags[i];
        if (nf & NF_REPLICA) continue;                     // counted by the owning rank
        int type = (int)(nf & NF_TYPE);
        double q = 0.0;
        bool flooded = false;
        if (type == OUTFALL) {
            double in = p.inflow[i], out = p.outflow[i];
            if (out == 0.0) q = in;
            else if (in == 0.0) {
                q = -out;
                p.inflow[i] = fabs(q);
            }
            p.overflow[i] = 0.0;
            p.nNewVolume[i] = 0.0;
        } else {
            if (p.nNewVolume[i] <= p.fullVolume[i]) q = p.overflow[i];
            if (q > 0.0) flooded = true;
        }
        if (q > 0.0) {
            if (flooded) acc[1] += q; else acc[0] += q;
        } else {
            acc[2] += -q;
        }
        const double newDepth = p.nNewDepth[i];
        if (type != OUTFALL && !steady)   // setNodeDepth's last dYdT (dynwave.c:750)
            p.dYdT[i] = fabs(newDepth - p.nOldDepth[i]) / dt;
        if (p.varStep && type != OUTFALL) {
            double y = newDepth;
            double yc = p.crownElev[i] - p.invert[i];
            if (!(y <= 0.0001) && !(y + 0.0001 >= yc)) {
                double maxDepth = yc * 0.25;
                double d = p.dYdT[i];
                if (!(maxDepth < 0.0001) && !(d < 0.0001)) {
                    double t1 = maxDepth / d;
                    if (t1 < acc[6]) { acc[6] = t1; acc[9] = (double)i; }
                }
            }
        }
        // per-node volume totals: the pending half step (state at the end of
        // the previous step) then this step's end state, each over dt/2
        double inflow = p.inflow[i], outflow = p.outflow[i], overflow = p.overflow[i];
        double newVolume = p.nNewVolume[i], fullVolume = p.fullVolume[i];
        if (!(p.endSkip & 8)) {
            double in = S.mbIn[i], out = S.mbOut[i];
            in += S.mbPendIn[i] * half;
            out += S.mbPendOut[i] * half;
            double ovfPrev = S.mbPendOut[p.nN + i];
            out += ovfPrev * half;
            double o1, o2;
            if (type == OUTFALL || (nf & NF_DEG0)) { o1 = inflow; o2 = 0.0; }
            else { o1 = outflow; o2 = (newVolume <= fullVolume) ? overflow : 0.0; }
            in += inflow * half;
            out += o1 * half;
            out += o2 * half;
            S.mbIn[i] = in;
            S.mbOut[i] = out;
            S.mbPendIn[i] = inflow;
            S.mbPendOut[i] = o1;
            S.mbPendOut[p.nN + i] = o2;
        }
        if (type == STORAGE) {                              // removeStorageLosses (routing.c:812-838)
            acc[3] += p.nEvapVol[i] / dt;
            acc[4] += p.nExfilVol[i] / dt;
        }
        if (!converged && !p.conv[i]) S.nonConv[i] += 1;  // stats_updateConvergenceStats
        if (!stats || (p.endSkip & 16)) continue;
        // stats_updateNodeStats (stats.c:543-643)
        S.avgDepth[i] += newDepth;
        if (newDepth > S.maxDepth[i]) { S.maxDepth[i] = newDepth; S.maxDepthDate[i] = aDate; }
        if (type != OUTFALL) {
            if (newVolume > fullVolume || overflow > 0.0) {
                S.timeFlooded[i] += dt;
                S.volFlooded[i] += overflow * dt;
                if (nf & NF_CANPOND) S.maxPonded[i] = gmax(S.maxPonded[i], (newVolume - fullVolume));
            }
            if ((type != STORAGE || p.surDepth[i] > 0.0) && newDepth + p.invert[i] + 0.0001 >= p.crownElev[i])
                S.timeSurch[i] += dt;
            if (type == STORAGE) {                         // stats.c:590-603
                S.sAvgVol[i] += newVolume;
                S.sEvap[i] += p.nEvapVol[i];
                S.sExfil[i] += p.nExfilVol[i];
                double v = gmin(newVolume, fullVolume);
                if (v > S.sMaxVol[i]) { S.sMaxVol[i] = v; S.sMaxVolDate[i] = aDate; }
                S.sMaxFlow[i] = gmax(S.sMaxFlow[i], outflow);
            }
        } else {
            if (inflow >= 0.001) {
                S.oAvgFlow[i] += inflow;
                S.oMaxFlow[i] = gmax(S.oMaxFlow[i], inflow);
                S.oPeriods[i] += 1;
            }
            for (int pp = 0; pp < p.P; pp++)                // this step's concentrations (k_qual_node)
                S.oLoad[(size_t)pp * p.nN + i] += inflow * p.nQual[c->qualPar ^ 1][(size_t)pp * p.nN + i] * dt;
            acc[7] += inflow;
        }
        double newLat = p.newLat[i];
        S.totLat[i] += ((p.oldLat[i] + newLat) * 0.5 * dt);
        if (fabs(newLat) > fabs(S.maxLat[i])) S.maxLat[i] = newLat;
        if (inflow > S.maxInflow[i]) { S.maxInflow[i] = inflow; S.maxInflowDate[i] = aDate; }
        if (overflow > S.maxOverflow[i]) { S.maxOverflow[i] = overflow; S.maxOverflowDate[i] = aDate; }
    }
    // wave reduction (fixed butterfly order), then wave partials in LDS
    int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int off = 32; off > 0; off >>= 1) {
        double o[kNumPartials];
        for (int q = 0; q < kNumPartials; q++) o[q] = __shfl_down(acc[q], off, 64);
        if (lane + off < 64) combinePartials(acc, o);
    }
    if (lane == 0)
        for (int q = 0; q < kNumPartials; q++) red[q][wv] = acc[q];
    __syncthreads();
    if (threadIdx.x == 0) {
        double v[kNumPartials];
        for (int q = 0; q < kNumPartials; q++) v[q] = red[q][0];
        for (int w = 1; w < kBlock / 64; w++) {
            double o[kNumPartials];
            for (int q = 0; q < kNumPartials; q++) o[q] = red[q][w];
            combinePartials(v, o);
        }
        for (int q = 0; q < kNumPartials; q++) p.partials[(size_t)blockIdx.x * kNumPartials + q] = v[q];
    }
}

// single-block finalisation (fixed-order reductions -> deterministic)
// kPhase 0: reduce + apply (one GPU).  Multi-GPU: phase 1 reduces this rank's
// partials into ctl->stepRed, the host/RCCL takes the min of the two Courant
// limits over the ranks, phase 2 applies.
template <int kPhase>
__global__ void k_finalize(Params p)
{
    __shared__ double sum[kNumPartials][kBlock];
    // the step-control block is staged through LDS: one coalesced load and
    // store instead of a chain of dependent single-lane HBM round trips
    __shared__ unsigned long long cw[sizeof(StepCtl) / 8];
    static_assert(sizeof(StepCtl) % 8 == 0, "StepCtl staged as 8-byte words");
    constexpr int nw = (int)(sizeof(StepCtl) / 8);
    int t = threadIdx.x;
    {
        const unsigned long long* g = (const unsigned long long*)p.ctl;
        for (int w = t; w < nw; w += kBlock) cw[w] = g[w];
    }
    StepCtl* c = (StepCtl*)cw;
    // Picard step count / convergence (dynwave.c:242-257): its flags load
    // alongside the partials
    bool converged = false;
    const int steps = (t == 0 && kPhase != 1) ? stepIterations(p, &converged) : 0;
    if (kPhase != 2) {
        double acc[kNumPartials];
        for (int q = 0; q < kNumPartials; q++) acc[q] = partialIsMin(q) || q == 8 || q == 9 ? 1.0e300 : 0.0;
        for (int b = t; b < p.nBlocksEnd; b += kBlock) {
            double v[kNumPartials];
            for (int q = 0; q < kNumPartials; q++) v[q] = p.partials[(size_t)b * kNumPartials + q];
            combinePartials(acc, v);
        }
        for (int q = 0; q < kNumPartials; q++) sum[q][t] = acc[q];
        __syncthreads();
        for (int h = kBlock / 2; h > 0; h >>= 1) {      // fixed-shape tree: deterministic
            if (t < h) {
                double a[kNumPartials], b[kNumPartials];
                for (int q = 0; q < kNumPartials; q++) { a[q] = sum[q][t]; b[q] = sum[q][t + h]; }
                combinePartials(a, b);
                for (int q = 0; q < kNumPartials; q++) sum[q][t] = a[q];
            }
            __syncthreads();
        }
        if (t == 0)
            for (int q = 0; q < kNumPartials; q++) c->stepRed[q] = sum[q][0];
        if (kPhase == 1 && t == 0 && p.skipSteady) {    // this rank's part of the step's flow totals
            const double* r = c->stepRed;
            const double s6[6] = {c->latTot[0], c->latTot[1] + r[2], r[1], c->latTot[2] + r[0], r[3], r[4]};
            for (int q = 0; q < 6; q++) c->steadyIO[q] = s6[q];
        }
    }
    __syncthreads();
    if (t == 0 && kPhase != 1) {
    double tot[kNumPartials];
    for (int q = 0; q < kNumPartials; q++) tot[q] = c->stepRed[q];
    // a step skipped as steady ran no Picard iteration (routing.c:239-244)
    const bool steady = p.skipSteady && c->steadyOk && !c->steadyChanged && !(c->steadyIO[6] > 0.0);
    const int ran = steady ? 0 : steps;
    c->lastSteps = ran;
    c->totalSteps += 1;
    if (p.P > 0) c->qualPar ^= 1;                      // this step's concentrations become the latest
    c->totalIters += ran;
    if (!converged && !steady) c->nonConverge += 1;
    // mass balance: massbal_updateRoutingTotals(dt/2) at both ends of the step
    double half = c->dt / 2.;
    double step[kNumPartials] = {c->latTot[0], c->latTot[1] + tot[2], tot[1], c->latTot[2] + tot[0],
                                 tot[3], tot[4], 0, 0};
    for (int q = 0; q < 6; q++) {
        c->flowTot[q] += c->prevStepTot[q] * half;
        c->flowTot[q] += step[q] * half;
        c->prevStepTot[q] = step[q];
    }
    // SKIP_STEADY_STATE: the next step may be steady when this step's flow
    // error (massbal_getStepFlowError, massbal.c:995-1017) is within
    // SYS_FLOW_TOL (isInSteadyState, routing.c:383-395; the next step's
    // OldRoutingTime is past 0); k_steady then checks the inflows
    if (p.skipSteady) {
        // several ranks: the totals summed over the ranks (k_finalize<1>,
        // then the exchange); the same decision on every rank
        const double* sv = (kPhase == 2) ? c->steadyIO : step;
        const double in = sv[0] + sv[1], out = sv[2] + sv[3] + sv[4] + sv[5];
        double err;
        if (fabs(in) > 0.0) err = 1.0 - out / in;
        else if (fabs(out) > 0.0) err = in / out - 1.0;
        else err = 0.0;
        c->steadyOk = fabs(err) <= p.sysFlowTol ? 1 : 0;
        c->steadyChanged = 0;
        c->steadyIO[6] = 0.0;
    }
    // run statistics of this step (routing.c:255-260): stats_updateFlowStats'
    // system part and stats_updateTimeStepStats (stats.c:449-518)
    {
        double dt = c->dt;
        double tEnd = c->newRoutingTime + 1000.0 * c->dt;
        double aDate = c->dateBase + (c->dateSecs0 + (tEnd + 1) / 1000.0) / 86400.0;
        if (!(aDate < c->statsStart)) {
            c->reportStepCount += 1;
            c->routingTimeSpan += dt;
            c->maxOutfallFlow = gmax(c->maxOutfallFlow, tot[7]);
        }
        if (steady) {
            c->tsSteadyTime += dt;
        } else {
            if (c->newRoutingTime > 0) {
                c->tsMin = gmin(c->tsMin, dt);
                for (int j = 1; j < kTimeLevels; j++)
                    if (dt >= c->tsIntervals[j]) { c->tsCounts[j] += 1; break; }
            }
            c->tsMax = gmax(c->tsMax, dt);
            c->tsRoutingTime += dt;
            c->tsCount += 1;
            c->tsTrials += steps;
        }
    }
    // advance the clock (routing.c:301-302)
    c->newRoutingTime = c->newRoutingTime + 1000.0 * c->dt;
    // step length of the next step: dynwave_getRoutingStep (dynwave.c:195-220,
    // 799-832) then execRouting's end-of-run clamp (swmm5.c:538-546)
    double dtn = c->routeStep;
    if (p.varStep && !c->varStepOff) {
        int crit = 0;
        double tMin = courantStep(tot[5], tot[6], c->routeStep, p.minRouteStep, &crit);
        // getVariableStep's critical element (dynwave.c:815-828) -- counted
        // when that next step will actually be routed (swmm5.c:531)
        if (!p.multi && c->newRoutingTime < c->routingDuration) {
            if (crit == 2) p.st.timeCourant[(int)tot[9]] += 1.0;
            else if (crit == 1) p.st.lTimeCourant[(int)tot[8]] += 1.0;
        }
        c->variableStep = tMin;
        dtn = c->variableStep;
    }
    c->dtNext = dtn;
    if (c->newRoutingTime + 1000.0 * dtn > c->routingDuration) {
        dtn = (c->routingDuration - c->newRoutingTime) / 1000.0;
        dtn = (dtn >= 1. / 1000.0) ? dtn : 1. / 1000.0;
    }
    c->dt = dtn;
    // next step's dt straight into host memory: the host clock advances
    // without a copy command in the step (totalSteps = index of that step)
    p.hostDt[c->totalSteps % kDtRing] = dtn;
    p.hostDt[kDtRing + (c->totalSteps - 1) % kDtRing] = (double)ran;     // Picard iterations of this step
    // nodes not frozen after iteration 1 (the sparse tail's live list): the
    // host's graph choice for the next steps
    p.hostDt[2 * kDtRing + 1 + (c->totalSteps - 1) % kDtRing] = tot[10];
    // a k_tail grid barrier that timed out (never expected: its workgroups
    // are co-resident by construction) is reported to the host at once
    p.hostDt[2 * kDtRing] = (double)c->tailErr;
    // No system-scope fence on the common path: the dt and iteration slots
    // are read after an event behind this step completed (launchedDt's
    // hipEventSynchronize, chooseGraph's hipEventQuery), and kernel
    // completion makes these host-memory writes visible.  The k_tail error
    // flag is also polled without an event (tailFailed): on that rare path
    // the write is pushed out at once
    if (c->tailErr) __threadfence_system();
    }
    if (c->tailErr)                                // leave no junction frozen in a failed step
        for (int i = t; i < p.nN; i += kBlock) p.frz[i] = 0;
    __syncthreads();
    if (kPhase != 1)                               // the next step's convergence flags
        for (int k = t; k < p.maxTrials; k += kBlock) p.unconv[k] = 0;
    if (kPhase != 1 && t == 0 && p.ipc && p.P > 0) // XCHG_IPC: this step's concentration exchange is complete
        p.xctl->qualSeq += 1;
    unsigned long long* g = (unsigned long long*)p.ctl;
    for (int w = t; w < nw; w += kBlock) g[w] = cw[w];
}

// Results of one reporting period (node_getResults node.c:497-528,
// link_getResults link.c:674-724, output.c:636-695): interpolation between the
// step's old and new state with weight f, converted to user units and packed
// as float32 in the .out variable order.  Host code writes the reported rows
// and sums the system storage from the same floats.
template <bool kFast>
__global__ __launch_bounds__(kBlock) void k_pack_results(Params p, double f, double uL, double uV,
                                                         double uQ, float* outN, float* outL)
{
    __shared__ double ct[kFast ? kCtFast : 5 * SWX_CIRC_N];
    stageTables(ct, p.gTables, kFast ? p.nGeom : 0);
    const double f1 = 1.0 - f;
    const int nv = 6 + p.P, lv = 5 + p.P;
    int n = gridDim.x * kBlock;
    for (int j = blockIdx.x * kBlock + threadIdx.x; j < p.nN; j += n) {
        float* x = outN + (size_t)j * nv;
        double z = (f1 * p.nOldDepth[j] + f * p.nNewDepth[j]) * uL;
        x[0] = (float)z;
        z = p.invert[j] * uL;
        x[1] = x[0] + (float)z;
        z = (f1 * p.nOldVolume[j] + f * p.nNewVolume[j]) * uV;
        x[2] = (float)z;
        z = (f1 * p.oldLat[j] + f * p.newLat[j]) * uQ;
        x[3] = (float)z;
        z = (f1 * p.oldFlowInflow[j] + f * p.inflow[j]) * uQ;
        x[4] = (float)z;
        z = p.overflow[j] * uQ;
        x[5] = (float)z;
        for (int q = 0; q < p.P; q++) {
            size_t k = (size_t)q * p.nN + j;
            z = f1 * p.nQual[p.ctl->qualPar ^ 1][k] + f * p.nQual[p.ctl->qualPar][k];
            x[6 + q] = (float)z;
        }
    }
    for (int j = blockIdx.x * kBlock + threadIdx.x; j < p.nL; j += n) {
        float* x = outL + (size_t)j * lv;
        uint32_t fl = p.lflags[j];
        Geom g = (fl & LF_COLD) ? loadGeom<false>(p, j, fl) : loadGeom<kFast>(p, j, fl, ct);
        double y = f1 * p.lOldDepth[j] + f * p.lNewDepth[j];
        double q = f1 * p.lOldFlow[j] + f * p.lNewFlow[j];
        double v = f1 * p.lOldVolume[j] + f * p.lNewVolume[j];
        double u = 0.0;
        double c = 0.0;
        if ((fl & LF_NC) && !(fl & LF_DUMMY)) {         // DUMMY conduits: u = c = 0 below
            c = p.setting[j];                            // link.c:699-707
            double qo = p.lOldFlow[j], qn = p.lNewFlow[j];
            if ((fl & LF_PUMP) && qo * qn == 0.0) q = (f >= f1) ? qn : qo;
        } else {
            if (y > 0.01) {                              // link_getVelocity link.c:821-843
                double barrels = (double)((fl >> LF_BARREL_SHIFT) & 0xFF);
                double fq = q / barrels;
                double area = getAofY(g, y, ct);
                if (area > 0.0001) u = fq / area;
            }
            if (g.type != G_DUMMY) c = getAofY(g, y, ct) / g.aFull;
        }
        double dir = (fl & LF_DIRNEG) ? -1.0 : 1.0;
        y *= uL;
        v *= uV;
        q *= uQ * dir;
        u *= uL * dir;
        x[0] = (float)q;
        x[1] = (float)y;
        x[2] = (float)u;
        x[3] = (float)v;
        x[4] = (float)c;
        for (int qq = 0; qq < p.P; qq++) {
            size_t k = (size_t)qq * p.nLs + j;
            c = f1 * p.lQual[p.ctl->qualPar ^ 1][k] + f * p.lQual[p.ctl->qualPar][k];
            x[5 + qq] = (float)c;
        }
    }
}

// REPORT AVERAGES: output_updateAvgResults (output.c:857-907) on the current
// results packed by k_pack_results with f = 1 (node_getResults(i, 1.0),
// link_getResults(i, 1.0)).  The sums are float32, as the reference's REAL4
// accumulators; a non-conduit link's capacity entry (pump speed, regulator
// opening) is not averaged: it holds the current value times the step count
// plus one, which the average returns.
__global__ __launch_bounds__(kBlock) void k_avg_accum(Params p, const float* resN, const float* resL,
                                                      float* avgN, float* avgL, float stepsPlus1)
{
    const size_t nv = (size_t)(6 + p.P), lv = (size_t)(5 + p.P);
    const size_t nN = (size_t)p.nN * nv, nL = (size_t)p.nL * lv, n = (size_t)gridDim.x * kBlock;
    for (size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x; t < nN; t += n) avgN[t] += resN[t];
    for (size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x; t < nL; t += n) {
        const size_t j = t / lv;
        const uint32_t fl = p.lflags[j];
        if (t - j * lv == 4 && (fl & LF_NC) && !(fl & LF_DUMMY)) avgL[t] = resL[t] * stepsPlus1;
        else avgL[t] += resL[t];
    }
}
// output_saveAvgResults (output.c:911-955): sum / Nsteps in float32, then the
// sums reset (output_initAvgResults, output.c:839-853)
__global__ __launch_bounds__(kBlock) void k_avg_take(size_t nN, size_t nL, float* avgN, float* avgL, float* outN,
                                                     float* outL, float steps)
{
    const size_t n = (size_t)gridDim.x * kBlock;
    for (size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x; t < nN; t += n) {
        outN[t] = avgN[t] / steps;
        avgN[t] = 0.0f;
    }
    for (size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x; t < nL; t += n) {
        outL[t] = avgL[t] / steps;
        avgL[t] = 0.0f;
    }
}

// ===========================================================================
//  Router implementation
// ===========================================================================
struct Router::Impl {
    Params p{};
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;      // fork/join branch for the cold conduits
    Partition part;                  // this rank's part of the network (whole net on one GPU)
    ncclComm_t comm = nullptr;       // RCCL communicator (multi-GPU, RCCL transport)
    int gridX = 1;                   // k_xpack / k_xunpack grid
    double* hostX = nullptr;         // host staging for the test transport
    std::vector<double> slotBuf;     // host transport: global ghost-slot buffer
    std::string xerrMsg;             // last failed collective / transfer
    // XCHG_IPC: this rank's uncached exchange region and the peers' regions
    // as mapped here (nullptr: self or unmapped); host-mapped failure record
    // and abort word; the transport actually in use (after any fallback)
    void* ipcBase = nullptr;
    std::vector<void*> ipcPeer;
    int* xerrHost = nullptr;
    int* hostAbortH = nullptr;
    double xTimeoutSec = 60.0;       // SWMM5_XCHG_TIMEOUT: bound of every wait behind an exchange
    // k_ipc_xchg (pack and unpack in one launch) instead of k_ipc_pack +
    // k_ipc_unpack: one kernel boundary less per exchange (tools/
    // ipc_signal_probe), but with ranks time-sharing one GPU its waiting
    // workgroups held the other rank's kernels back (147 against 17 us per
    // exchange).  So it is chosen when every rank drives
    // a GPU of its own (setupIpc compares the ranks' PCI addresses);
    // SWMM5_XCHG_FUSED=0/1 forces either
    bool xchgFused = false;
    int xchgFusedEnv = -1;
    std::string transportName = "single";
    float *resN = nullptr, *resL = nullptr;          // packed period results (device)
    float *resNHost = nullptr, *resLHost = nullptr;  // pinned copies
    float *avgN = nullptr, *avgL = nullptr;          // REPORT AVERAGES: the period's sums
    float *avgON = nullptr, *avgOL = nullptr;        // and its averages (device)
    float *avgONHost = nullptr, *avgOLHost = nullptr;
    double* depthHost = nullptr;
    int avgSteps = 0;                                // output.c Nsteps
    std::vector<hipEvent_t> forkEv, joinEv;   // per Picard iteration (cold-conduit fork / join)
    hipGraphExec_t graph = nullptr;
    // step graph whose iterations k >= 2 run in k_tail (Router::step picks
    // it or the unrolled graph: SWMM5_TAIL = 0 never, 1 always, else auto)
    hipGraphExec_t graphTail = nullptr;
    int tailMode = 2;
    int tailGrid = 0;
    double itersAvg = 0.0;           // moving average of Picard iterations per step
    long long itersSeen = -1;        // last step whose count was read from hostDt
    // step graph whose iterations k >= 2 run in k_sparse (one workgroup) and
    // k_unfreeze: SWMM5_SPARSE = 0 never, 1 always, else auto (live lists of
    // at most sparseMax nodes)
    hipGraphExec_t graphSparse = nullptr;
    int sparseMode = 2;
    bool sparseOk = false;
    // the list graph: at least three iterations; partitioned runs and
    // networks with pumps / regulators too (its iterations carry the
    // neighbour exchange, k_nc and the flag all-reduce as the unrolled
    // graph's do)
    bool listOk = false;
    double sparseMax = 6000.0;
    double liveAvg = 0.0;            // moving average of the live-list length after iteration 1
    long long modeSteps[4] = {0, 0, 0, 0};   // steps launched per graph (unrolled, k_tail, sparse, list)
    hipGraphExec_t graphList = nullptr;   // iterations k >= 2 as list-driven k_walk / k_node_list pairs
    double listMax = 200000.0;       // auto: the list graph while the live lists average at most this
    bool useGraph = true;
    bool timing = false;
    int gridL = 1, gridN = 1, gridEnd = 1, gridC = 1;
    int gridQ = 1;                   // k_qual_node grid
    int gridLinkSparse = 1;          // k_link grid of iterations k >= 2 (unconverged-list walk)
    bool fuseQual = false;           // quality in the step-end kernel (k_step_end<..., kQual>)
    int gridNList = 1;               // k_node_list grid (list graph)
    int linkWaves = kLinkWavesDefault;
    bool fastLinks = false;          // all streaming conduits circular, no SLOT
    bool general = false;            // storage units or non-basic shapes (k_node/k_step_end<.., true>)
    bool allShapes = false;          // non-basic conduit shapes present
    std::vector<void*> allocs;
    double* latBase = nullptr;       // constant lateral inflows
    double* qualBase = nullptr;
    double* hostPinned = nullptr;    // staging for uploads
    size_t pinnedSize = 0;
    StepCtl* ctl = nullptr;
    StepCtl* hostCtl = nullptr;      // pinned
    bool constantInflow = true;
    struct TimingSlot {               // one timed step's events + readback
        std::vector<hipEvent_t> ev, evHot;
        std::vector<hipEvent_t> evX;  // several ranks: per iteration [4k, 4k+1] ghost exchange, [4k+2, 4k+3] flag
        unsigned long long* pinned = nullptr;   // [0] iterations run, [1..] conduits updated, nodes gathered
        int mode = 0;                 // graph the step mirrored (0 unrolled, 2 sparse: k >= 2 in k_sparse)
    };
    std::vector<TimingSlot> tslots;
    double climateDev[3] = {0, 0, 0}; // StepCtl::evapRate, hydconFactor, recoveryFactor on the device
    double* evapPinned = nullptr;      // pinned ring of those for setClimate's async copies
    hipEvent_t evapEv[kDtRing] = {};
    int evapNext = 0;
    std::vector<double> probeSum;     // SWMM5_PROBE: [k][kProbeSlots + 1] phase microseconds, count
    double wallKHz = 100000.0;
    int tUsed = 0;
    hipEvent_t* curEv = nullptr;     // event set of the step being launched
    hipEvent_t* curHot = nullptr;
    hipEvent_t* curX = nullptr;      // evX of the step being launched (null: not timed)
    // kernel classes: 0 k_link<first>, 1 k_node<first>, 2 step end (k_step_end +
    // k_finalize), 3 quality, 4 k_link iterations >= 1, 5 k_node iteration 1,
    // 6 k_node iterations >= 2, 7 k_sparse + k_unfreeze (iterations >= 2 of a
    // sparse-graph step)
    // 8 ghost-link exchange (pack .. unpack, every iteration), 9 convergence
    // flag exchange (several ranks only)
    static constexpr int kClasses = 10;
    long long itersTimed1 = 0;        // timed iterations k >= 1 that ran (either graph)
    double kms[kClasses] = {};
    long long kcnt[kClasses] = {};
    double kbytes[kClasses] = {};     // byte model per launch (class 4: per updated conduit)
    double kbytesSum[kClasses] = {};  // algorithmic bytes of the timed launches
    // node byte model: iteration 1 per launch; iterations >= 2 per scanned node,
    // per relaxation-only update, per full update and per gathering node
    double nodeIter1 = 0, nodeScan = 0, nodeFastB = 0, nodeUpdB = 0, nodeGather = 0;
    double gatherSum = 0, gatherCnt = 0;  // nodes gathered at iterations >= 2
    double nHot = 0, nColdD = 0;
    double workSum = 0;               // conduits updated in timed iterations >= 1
    // per Picard iteration k of the timed steps: [0] launches, [1] conduits
    // updated, [2] nodes gathered, [3] nodes updated (not frozen), [4]
    // relaxation-only node updates, [5] k_link ms, [6] k_node ms
    static constexpr int kIterCols = 7;
    std::vector<double> iterStats;
    int nE = 0;
    bool tableShapes = true;
    static constexpr int kRing = kDtRing;
    hipEvent_t ringEv[kRing] = {};
    hipEvent_t clockEv[kRing] = {};  // completion of step n -> clockEv[n % kRing]
    double* hostDt = nullptr;        // host-mapped ring: dt of step n in slot n % kRing
    long long launched = 0;          // steps passed to step()
    int ringNext = 0;
    size_t slotDoubles = 0;
    double lastDtHost = 0.0;
    double latTot0[3] = {0, 0, 0};
};

Router::Router() : d_(new Impl) {}
Router::~Router()
{
    if (d_) {
        if (d_->graph) (void)hipGraphExecDestroy(d_->graph);
        if (d_->graphTail) (void)hipGraphExecDestroy(d_->graphTail);
        if (d_->graphSparse) (void)hipGraphExecDestroy(d_->graphSparse);
        if (d_->graphList) (void)hipGraphExecDestroy(d_->graphList);
        for (auto& t : d_->tslots) {
            for (auto e : t.ev) (void)hipEventDestroy(e);
            for (auto e : t.evHot) (void)hipEventDestroy(e);
            for (auto e : t.evX) (void)hipEventDestroy(e);
            if (t.pinned) (void)hipHostFree(t.pinned);
        }
        for (void* a : d_->allocs) (void)hipFree(a);
        if (d_->hostPinned) (void)hipHostFree(d_->hostPinned);
        if (d_->hostCtl) (void)hipHostFree(d_->hostCtl);
        if (d_->hostDt) (void)hipHostFree(d_->hostDt);
        if (d_->hostX) (void)hipHostFree(d_->hostX);
        if (d_->resNHost) (void)hipHostFree(d_->resNHost);
        if (d_->resLHost) (void)hipHostFree(d_->resLHost);
        if (d_->avgONHost) (void)hipHostFree(d_->avgONHost);
        if (d_->avgOLHost) (void)hipHostFree(d_->avgOLHost);
        if (d_->depthHost) (void)hipHostFree(d_->depthHost);
        if (d_->comm) (void)ncclCommDestroy(d_->comm);
        for (void* q : d_->ipcPeer)
            if (q) (void)hipIpcCloseMemHandle(q);
        if (d_->ipcBase) (void)hipFree(d_->ipcBase);
        if (d_->xerrHost) (void)hipHostFree(d_->xerrHost);
        if (d_->hostAbortH) (void)hipHostFree(d_->hostAbortH);
        for (auto e : d_->clockEv) if (e) (void)hipEventDestroy(e);
        for (auto e : d_->evapEv) if (e) (void)hipEventDestroy(e);
        if (d_->evapPinned) (void)hipHostFree(d_->evapPinned);
        for (auto e : d_->ringEv) if (e) (void)hipEventDestroy(e);
        for (auto e : d_->forkEv) if (e) (void)hipEventDestroy(e);
        for (auto e : d_->joinEv) if (e) (void)hipEventDestroy(e);
        if (d_->side) (void)hipStreamDestroy(d_->side);
        if (d_->stream) (void)hipStreamDestroy(d_->stream);
        delete d_;
    }
}

template <class T>
static T* devAlloc(Router::Impl* d, size_t n, hipError_t* err)
{
    void* ptr = nullptr;
    *err = hipMalloc(&ptr, std::max<size_t>(n, 1) * sizeof(T));
    if (*err == hipSuccess) d->allocs.push_back(ptr);
    return (T*)ptr;
}

typedef void (*LinkKernelFn)(Params, int);
template <bool kFast>
static LinkKernelFn linkKernelT(bool first, int waves)
{
    switch (waves) {
    case 3: return first ? k_link<true, 3, kFast> : k_link<false, 3, kFast>;
    case 4: return first ? k_link<true, 4, kFast> : k_link<false, 4, kFast>;
    default: return first ? k_link<true, 1, kFast> : k_link<false, 1, kFast>;
    }
}
static LinkKernelFn linkKernel(bool first, int waves, bool fast)
{
    return fast ? linkKernelT<true>(first, waves) : linkKernelT<false>(first, waves);
}
typedef void (*StepEndFn)(Params);
static StepEndFn stepEndKernel(bool fast, bool all, bool qual = false)
{
    if (qual) {
        if (fast) return all ? k_step_end<true, true, true> : k_step_end<true, false, true>;
        return all ? k_step_end<false, true, true> : k_step_end<false, false, true>;
    }
    if (fast) return all ? k_step_end<true, true> : k_step_end<true, false>;
    return all ? k_step_end<false, true> : k_step_end<false, false>;
}
static LinkKernelFn nodeKernel(bool first, bool storage)
{
    if (storage) return first ? k_node<true, true> : k_node<false, true>;
    return first ? k_node<true, false> : k_node<false, false>;
}

// ---- multi-GPU collectives ------------------------------------------------
// Every call returns 0 or 500 with d->xerrMsg set.  On the RCCL transport the
// calls are enqueued on the routing stream (captured into the step graph at
// init, where a failing call fails Router::init); the host transport (tests:
// gloo through a callback) runs them synchronously.
static int xfail(Router::Impl* d, const std::string& what)
{
    d->xerrMsg = what;
    return 500;
}
static int ncclCheck(Router::Impl* d, ncclResult_t r, const char* what)
{
    if (r == ncclSuccess) return 0;
    return xfail(d, std::string(what) + ": " + ncclGetErrorString(r));
}
static int hipCheckX(Router::Impl* d, hipError_t e, const char* what)
{
    if (e == hipSuccess) return 0;
    return xfail(d, std::string(what) + ": " + hipGetErrorString(e));
}
// host transport: in-place reduction of n doubles over the ranks
static int hostReduce(Router::Impl* d, double* buf, long n, int op)
{
    if (!d->part.xchg) return xfail(d, "host exchange callback missing");
    if (d->part.xchg(buf, n, op, d->part.xuser)) return xfail(d, "host exchange callback failed");
    return 0;
}

// XCHG_IPC: the device's failure record as a message; false when there is none
static bool ipcFailed(Router::Impl* d, std::string* msg)
{
    if (!d->xerrHost) return false;
    const int code = __atomic_load_n(&d->xerrHost[0], __ATOMIC_ACQUIRE);
    if (!code) return false;
    static const char* kinds[] = {"?", "ghost-link", "concentration", "convergence-flag", "reduction",
                                  "start-up handshake"};
    const int kind = d->xerrHost[1];
    const char* kn = (kind >= 0 && kind <= XK_HELLO) ? kinds[kind] : "?";
    char buf[320];
    if (code == 2)
        snprintf(buf, sizeof buf, "multi-GPU exchange aborted on rank %d: another rank gave up waiting "
                 "(%s exchange %d); the run is stopped on every rank", d->part.rank, kn, d->xerrHost[3]);
    else
        snprintf(buf, sizeof buf, "multi-GPU exchange timed out: rank %d waited more than %.0f s for rank %d "
                 "(%s exchange %d); every rank was told to stop", d->part.rank, d->xTimeoutSec,
                 d->xerrHost[2], kn, d->xerrHost[3]);
    *msg = buf;
    if (d->hostAbortH) __atomic_store_n(d->hostAbortH, 1, __ATOMIC_RELEASE);   // later waits exit at once
    return true;
}

// Bounded host waits (every synchronisation of the routing stream or of a
// step's completion event goes through here).  RCCL: the stream or event is
// polled together with the communicator's asynchronous error against a
// deadline (SWMM5_XCHG_TIMEOUT, default 60 s); on an RCCL error or at the
// deadline the communicator is aborted (ncclCommAbort makes its kernels
// return) and the router fails with error 500 instead of hanging.  IPC: the
// device's own waits are bounded; past the deadline the host also sets the
// host-mapped abort word every device wait polls.  The device's failure
// record is checked after every wait.
static int waitDone(Router::Impl* d, hipEvent_t ev)
{
    hipError_t e;
    const bool bounded = d->part.active() && (d->comm || d->part.transport == XCHG_IPC);
    if (bounded) {
        const auto t0 = std::chrono::steady_clock::now();
        bool hostAborted = false;
        for (;;) {
            e = ev ? hipEventQuery(ev) : hipStreamQuery(d->stream);
            if (e != hipErrorNotReady) break;
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (d->comm) {
                ncclResult_t as = ncclSuccess;
                if (ncclCommGetAsyncError(d->comm, &as) == ncclSuccess && as != ncclSuccess && as != ncclInProgress) {
                    (void)ncclCommAbort(d->comm);
                    d->comm = nullptr;
                    return xfail(d, std::string("RCCL asynchronous error: ") + ncclGetErrorString(as) +
                                        "; communicator aborted");
                }
                if (s > d->xTimeoutSec) {
                    (void)ncclCommAbort(d->comm);
                    d->comm = nullptr;
                    char buf[160];
                    snprintf(buf, sizeof buf, "an RCCL collective did not complete within %.0f s on rank %d; "
                             "communicator aborted", d->xTimeoutSec, d->part.rank);
                    return xfail(d, buf);
                }
            } else if (!hostAborted && s > d->xTimeoutSec + 5.0) {
                __atomic_store_n(d->hostAbortH, 1, __ATOMIC_RELEASE);
                hostAborted = true;
            } else if (hostAborted && s > 2.0 * d->xTimeoutSec + 10.0) {
                return xfail(d, "multi-GPU exchange: the device did not stop after the host abort");
            }
            usleep(20);
        }
    } else {
        e = ev ? hipEventSynchronize(ev) : hipStreamSynchronize(d->stream);
    }
    if (e != hipSuccess) return xfail(d, std::string("synchronisation: ") + hipGetErrorString(e));
    std::string m;
    if (ipcFailed(d, &m)) return xfail(d, m);
    return 0;
}

// In-place all-reduce of n doubles (op 0 sum, 1 min) -- the Courant limits.
static int exchange(Router::Impl* d, const double* send, double* recv, size_t n, int op)
{
    if (d->part.transport == XCHG_IPC) {
        if (send != recv || n > (size_t)kRedMax) return xfail(d, "IPC reduction: in place, at most 8 values");
        hipLaunchKernelGGL(k_ipc_reduce, dim3(1), dim3(64), 0, d->stream, d->p, recv, (int)n, op);
        return 0;
    }
    if (d->part.transport == XCHG_RCCL)
        return ncclCheck(d, ncclAllReduce(send, recv, n, ncclDouble, op ? ncclMin : ncclSum, d->comm, d->stream),
                         "ncclAllReduce");
    if (int r = hipCheckX(d, hipMemcpyAsync(d->hostX, send, n * sizeof(double), hipMemcpyDeviceToHost, d->stream),
                          "exchange D2H")) return r;
    if (int r = hipCheckX(d, hipStreamSynchronize(d->stream), "exchange sync")) return r;
    if (int r = hostReduce(d, d->hostX, (long)n, op)) return r;
    return hipCheckX(d, hipMemcpyAsync(recv, d->hostX, n * sizeof(double), hipMemcpyHostToDevice, d->stream),
                     "exchange H2D");
}

// Neighbour exchange of f doubles per link: xsend (packed, neighbour-major)
// to the ranks holding them as ghosts, xrecv (ghost order) from them.  RCCL:
// one grouped ncclSend / ncclRecv per neighbour (strip neighbours for the
// grids), no collective.  Host transport: every sent link has one global
// slot; each rank writes its links' slots and a sum over the ranks leaves
// every slot holding its owner's values exactly (x + 0.0 == x; a -0.0 becomes
// +0.0, which no node sum can tell apart).
static int neighbourExchange(Router::Impl* d, int f)
{
    const Partition& part = d->part;
    const Params& p = d->p;
    if (part.transport == XCHG_RCCL) {
        if (int r = ncclCheck(d, ncclGroupStart(), "ncclGroupStart")) return r;
        for (size_t k = 0; k < part.nbr.size(); k++) {
            const int ns = part.sendOff[k + 1] - part.sendOff[k], nr = part.recvOff[k + 1] - part.recvOff[k];
            if (ns > 0 && ncclCheck(d, ncclSend(p.xsend + (size_t)f * part.sendOff[k], (size_t)f * ns, ncclDouble,
                                                part.nbr[k], d->comm, d->stream), "ncclSend")) {
                (void)ncclGroupEnd();
                return 500;
            }
            if (nr > 0 && ncclCheck(d, ncclRecv(p.xrecv + (size_t)f * part.recvOff[k], (size_t)f * nr, ncclDouble,
                                                part.nbr[k], d->comm, d->stream), "ncclRecv")) {
                (void)ncclGroupEnd();
                return 500;
            }
        }
        return ncclCheck(d, ncclGroupEnd(), "ncclGroupEnd");
    }
    const size_t ns = part.sendLink.size(), ng = part.lghost.size(), slots = (size_t)f * part.nSlotGlobal;
    std::vector<double>& g = d->slotBuf;
    g.assign(slots, 0.0);
    if (ns) {
        if (int r = hipCheckX(d, hipMemcpyAsync(d->hostX, p.xsend, (size_t)f * ns * sizeof(double),
                                                hipMemcpyDeviceToHost, d->stream), "neighbour D2H")) return r;
        if (int r = hipCheckX(d, hipStreamSynchronize(d->stream), "neighbour sync")) return r;
        for (size_t e = 0; e < ns; e++)
            for (int q = 0; q < f; q++) g[(size_t)f * part.sendSlot[e] + q] = d->hostX[(size_t)f * e + q];
    }
    if (slots && hostReduce(d, g.data(), (long)slots, 0)) return 500;
    if (ng) {
        for (size_t e = 0; e < ng; e++)
            for (int q = 0; q < f; q++) d->hostX[(size_t)f * e + q] = g[(size_t)f * part.recvSlot[e] + q];
        if (int r = hipCheckX(d, hipMemcpyAsync(p.xrecv, d->hostX, (size_t)f * ng * sizeof(double),
                                                hipMemcpyHostToDevice, d->stream), "neighbour H2D")) return r;
        if (int r = hipCheckX(d, hipStreamSynchronize(d->stream), "neighbour sync")) return r;
    }
    return 0;
}

// Iteration k's "some node did not converge" flag, max over the ranks (in
// place in the per-iteration flags), so every rank runs the same iterations.
static int flagExchangeImpl(Router::Impl* d, int k);
static int flagExchange(Router::Impl* d, int k)
{
    if (d->curX) (void)hipEventRecord(d->curX[4 * k + 2], d->stream);
    const int r = flagExchangeImpl(d, k);
    if (d->curX) (void)hipEventRecord(d->curX[4 * k + 3], d->stream);
    return r;
}
static int flagExchangeImpl(Router::Impl* d, int k)
{
    int* flag = d->p.unconv + k;
    if (d->part.transport == XCHG_IPC) {
        hipLaunchKernelGGL(k_ipc_flag<false>, dim3(1), dim3(64), 0, d->stream, d->p, k, (int*)nullptr);
        return 0;
    }
    if (d->part.transport == XCHG_RCCL)
        return ncclCheck(d, ncclAllReduce(flag, flag, 1, ncclInt32, ncclMax, d->comm, d->stream), "ncclAllReduce");
    int v = 0;
    if (int r = hipCheckX(d, hipMemcpyAsync(&v, flag, sizeof(int), hipMemcpyDeviceToHost, d->stream), "flag D2H"))
        return r;
    if (int r = hipCheckX(d, hipStreamSynchronize(d->stream), "flag sync")) return r;
    double x = v ? 1.0 : 0.0;
    if (int r = hostReduce(d, &x, 1, 0)) return r;
    v = x > 0.0 ? 1 : 0;
    if (int r = hipCheckX(d, hipMemcpyAsync(flag, &v, sizeof(int), hipMemcpyHostToDevice, d->stream), "flag H2D"))
        return r;
    return hipCheckX(d, hipStreamSynchronize(d->stream), "flag sync");
}

// Iteration k's ghost-link values from their owners (before the node update):
// pack, transfer, unpack on the RCCL / host transports; on XCHG_IPC the owners
// store them straight into this rank's ghost area and k_ipc_unpack waits for
// them.  qualExchange: the ghost links' concentrations, once per step.
// Grid of a kernel that waits for the peers (k_ipc_unpack): at most
// kXchgGrid workgroups, so that its waiting waves never fill the GPU -- with
// several ranks on one device a full-grid waiter kept the peer's own kernels
// off the CUs it was waiting for (a 2-rank run with 4-row node blocks timed
// out) -- and no more than the ghosts need
static int waitGrid(const Router::Impl* d)
{
    const int need = (d->p.nGhost + kBlock - 1) / kBlock;
    return std::max(1, std::min(std::min(d->gridX, kXchgGrid), need));
}
static int ghostExchangeImpl(Router::Impl* d, int k);
static int ghostExchange(Router::Impl* d, int k)
{
    // timing mode: the exchange's span on the routing stream
    if (d->curX) (void)hipEventRecord(d->curX[4 * k], d->stream);
    const int r = ghostExchangeImpl(d, k);
    if (d->curX) (void)hipEventRecord(d->curX[4 * k + 1], d->stream);
    return r;
}
static int ghostExchangeImpl(Router::Impl* d, int k)
{
    const Params& p = d->p;
    if (d->part.transport == XCHG_IPC) {
        if (p.nSend && p.nGhost && d->xchgFused)
            hipLaunchKernelGGL(k_ipc_xchg<false>, dim3(kXchgGrid), dim3(kBlock), 0, d->stream, p, k);
        else {
            if (p.nSend) hipLaunchKernelGGL(k_ipc_pack<false>, dim3(d->gridX), dim3(kBlock), 0, d->stream, p, k);
            if (p.nGhost) hipLaunchKernelGGL(k_ipc_unpack<false>, dim3(waitGrid(d)), dim3(kBlock), 0, d->stream, p, k);
        }
        return 0;
    }
    if (p.nSend) hipLaunchKernelGGL(k_xpack, dim3(d->gridX), dim3(kBlock), 0, d->stream, p, k);
    if (int r = neighbourExchange(d, p.xF)) return r;
    if (p.nGhost) hipLaunchKernelGGL(k_xunpack, dim3(d->gridX), dim3(kBlock), 0, d->stream, p, k);
    return 0;
}
static int qualExchange(Router::Impl* d)
{
    const Params& p = d->p;
    if (d->part.transport == XCHG_IPC) {
        if (p.nSend && p.nGhost && d->xchgFused)
            hipLaunchKernelGGL(k_ipc_xchg<true>, dim3(kXchgGrid), dim3(kBlock), 0, d->stream, p, 0);
        else {
            if (p.nSend) hipLaunchKernelGGL(k_ipc_pack<true>, dim3(d->gridX), dim3(kBlock), 0, d->stream, p, 0);
            if (p.nGhost) hipLaunchKernelGGL(k_ipc_unpack<true>, dim3(waitGrid(d)), dim3(kBlock), 0, d->stream, p, 0);
        }
        return 0;
    }
    if (p.nSend) hipLaunchKernelGGL(k_xpack_qual, dim3(d->gridX), dim3(kBlock), 0, d->stream, p);
    if (int r = neighbourExchange(d, p.P)) return r;
    if (p.nGhost) hipLaunchKernelGGL(k_xunpack_qual, dim3(d->gridX), dim3(kBlock), 0, d->stream, p);
    return 0;
}

// Timing mode (eager launches, Router::setTiming): the link and node kernels
// of iteration k, the quality kernel and the step-end pair are launched with
// hipExtLaunchKernelGGL, whose start/stop events carry the kernels' own
// execution timestamps (the durations rocprofv3's kernel trace reports), not
// the dispatch gaps around them.  Events per step: [4k] / hot[k] k_link(k),
// [4k+1] / [4k+2] k_node(k), [base] / [base+1] quality, [base+2] / [base+3]
// k_step_end .. k_finalize (base = 4 MaxTrials).
template <typename F, typename... A>
static void launchTimedB(Router::Impl* d, F kernel, dim3 grid, dim3 block, hipEvent_t start, hipEvent_t stop,
                         A... args)
{
    if (d->timing)
        hipExtLaunchKernelGGL(kernel, grid, block, 0, d->stream, start, stop, 0, args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, 0, d->stream, args...);
}
template <typename F, typename... A>
static void launchTimed(Router::Impl* d, F kernel, dim3 grid, hipEvent_t start, hipEvent_t stop, A... args)
{
    launchTimedB(d, kernel, grid, dim3(kBlock), start, stop, args...);
}

// One Picard iteration k.  Conduits with an invert offset (k_link_cold) run on
// a side stream, concurrently with the streaming kernel, and are joined before
// the node update; without such conduits the iteration is two kernels on one
// stream (a cross-queue dependency costs ~5-10 us on MI355X, more than the
// cold work it would hide):
//   main:  [fork k] k_link(k) ─wait join k─ k_node(k)
//   side:  wait fork k ─ k_link_cold(k) ─[join k]
// Multi-GPU: k_link ─ k_xpack ─ neighbour send/recv ─ k_xunpack ─ k_node ─
// [k_nc] ─ all-reduce(max) of the iteration's convergence flag.
static int launchIteration(Router::Impl* d, int k)
{
    Params& p = d->p;
    const bool multi = d->part.active();
    if (p.nCold) {
        (void)hipEventRecord(d->forkEv[k], d->stream);
        (void)hipStreamWaitEvent(d->side, d->forkEv[k], 0);
        if (k == 0)
            hipLaunchKernelGGL(k_link_cold<true>, dim3(d->gridC), dim3(kBlock), 0, d->side, p, k);
        else
            hipLaunchKernelGGL(k_link_cold<false>, dim3(d->gridC), dim3(kBlock), 0, d->side, p, k);
        (void)hipEventRecord(d->joinEv[k], d->side);
    }
    hipEvent_t e0 = d->timing ? d->curEv[4 * k] : nullptr, e1 = d->timing ? d->curHot[k] : nullptr;
    if (k >= 2 && p.deferPro)                      // the walk with the deferred outfall work
        launchTimed(d, d->fastLinks ? k_walk<true, false, true> : k_walk<false, false, true>,
                    dim3(d->gridLinkSparse), e0, e1, p, k);
    else
        launchTimed(d, linkKernel(k == 0, d->linkWaves, d->fastLinks), dim3(k >= 2 ? d->gridLinkSparse : d->gridL),
                    e0, e1, p, k);
    if (p.nCold) (void)hipStreamWaitEvent(d->stream, d->joinEv[k], 0);
    if (multi)                                     // ghost links' values from their owners
        if (int r = ghostExchange(d, k)) return r;
    e0 = d->timing ? d->curEv[4 * k + 1] : nullptr;
    e1 = d->timing ? d->curEv[4 * k + 2] : nullptr;
    launchTimed(d, nodeKernel(k == 0, d->general), dim3(d->gridN), e0, e1, p, k);
    if (p.nNC > 0) {                               // pumps / regulators, their end nodes
        if (k == 0) hipLaunchKernelGGL(k_nc<true>, dim3(1), dim3(kBlock), 0, d->stream, p, k);
        else hipLaunchKernelGGL(k_nc<false>, dim3(1), dim3(kBlock), 0, d->stream, p, k);
    }
    if (multi) return flagExchange(d, k);
    return 0;
}

typedef void (*TailFn)(Params);
static TailFn tailKernel(bool fast, bool general)
{
    if (fast) return general ? k_tail<true, true> : k_tail<true, false>;
    return general ? k_tail<false, true> : k_tail<false, false>;
}

static TailFn sparseKernel(bool fast, bool general)
{
    if (fast) return general ? k_sparse<true, true> : k_sparse<true, false>;
    return general ? k_sparse<false, true> : k_sparse<false, false>;
}

// The step's launches.  GM_UNROLLED: every iteration k < MaxTrials as a
// k_link / k_node pair (later ones exit at once after convergence); GM_TAIL:
// iterations k >= 2 in one k_tail launch (d->tailGrid > 0 only); GM_SPARSE:
// iterations k >= 2 in k_sparse (one workgroup), then k_unfreeze
// (d->sparseOk only); GM_LIST: iterations k >= 2 as list-driven k_walk /
// k_node_list pairs, then k_unfreeze (d->listOk only).  (The round-4 fused
// and round-5 compact graphs were measured slower than the list graph and
// removed in round 6: DESIGN section 4.)
enum { GM_UNROLLED = 0, GM_TAIL = 1, GM_SPARSE = 2, GM_LIST = 3 };
static int launchStepImpl(Router::Impl* d, int mode);
static int launchStep(Router::Impl* d, int mode = GM_UNROLLED)
{
    // (each captured graph keeps its own copy of the arguments)
    Params& p = d->p;
    // the list graph with a separate quality launch: k_qual_node gives the
    // frozen junctions their final depth (each node's own thread, before its
    // quality reads the depth), one full-grid k_unfreeze less
    p.qualUnfreeze = (mode == GM_LIST && p.P > 0 && !d->fuseQual && p.freeze) ? 1 : 0;
    const int r = launchStepImpl(d, mode);
    p.qualUnfreeze = 0;
    return r;
}
static int launchStepImpl(Router::Impl* d, int mode)
{
    Params& p = d->p;
    // k_node(1) lists the live nodes only for the list-driven graphs
    p.buildVlist = (mode == GM_SPARSE || mode == GM_LIST) ? 1 : 0;
    const bool multi = d->part.active();
    if (p.skipSteady) {                            // SKIP_STEADY_STATE: this step's inflow test
        hipLaunchKernelGGL(k_steady, dim3(d->gridN), dim3(kBlock), 0, d->stream, p);
        if (multi)                                 // any rank's change makes the step routed everywhere
            if (int r = exchange(d, &p.ctl->steadyIO[6], &p.ctl->steadyIO[6], 1, 0)) return r;
    }
    const int base = 4 * p.maxTrials;
    hipEvent_t* ev = d->timing ? d->curEv : nullptr;
    if (mode == GM_TAIL) {
        for (int k = 0; k < 2; k++)
            if (int r = launchIteration(d, k)) return r;
        hipLaunchKernelGGL(tailKernel(d->fastLinks, d->general), dim3(d->tailGrid), dim3(kBlock), 0, d->stream, p);
    } else if (mode == GM_SPARSE) {
        for (int k = 0; k < 2; k++)
            if (int r = launchIteration(d, k)) return r;
        launchTimedB(d, sparseKernel(d->fastLinks, d->general), dim3(1), dim3(kSparseBlock),
                     ev ? ev[base + 4] : nullptr, (hipEvent_t) nullptr, p);
        launchTimed(d, k_unfreeze, dim3(d->gridN), (hipEvent_t) nullptr, ev ? ev[base + 5] : nullptr, p);
    } else if (mode == GM_LIST) {
        for (int k = 0; k < 2; k++)
            if (int r = launchIteration(d, k)) return r;
        for (int k = 2; k < p.maxTrials; k++) {
            if (p.nCold) {
                (void)hipEventRecord(d->forkEv[k], d->stream);
                (void)hipStreamWaitEvent(d->side, d->forkEv[k], 0);
                hipLaunchKernelGGL((k_link_cold<false>), dim3(d->gridC), dim3(kBlock), 0, d->side, p, k);
                (void)hipEventRecord(d->joinEv[k], d->side);
            }
            // the unrolled graph's walk: k_node_list finds the woken junctions
            // itself (no wake list)
            if (p.deferPro)
                launchTimed(d, d->fastLinks ? k_walk<true, false, true> : k_walk<false, false, true>,
                            dim3(d->gridLinkSparse), ev ? ev[4 * k] : nullptr, d->timing ? d->curHot[k] : nullptr, p, k);
            else
                launchTimed(d, linkKernel(false, d->linkWaves, d->fastLinks), dim3(d->gridLinkSparse),
                            ev ? ev[4 * k] : nullptr, d->timing ? d->curHot[k] : nullptr, p, k);
            if (p.nCold) (void)hipStreamWaitEvent(d->stream, d->joinEv[k], 0);
            if (multi)                             // ghost links' values from their owners (as launchIteration)
                if (int r = ghostExchange(d, k)) return r;
            launchTimed(d, d->general ? k_node_list<true> : k_node_list<false>, dim3(d->gridNList),
                        ev ? ev[4 * k + 1] : nullptr, ev ? ev[4 * k + 2] : nullptr, p, k);
            // pumps / regulators and their end nodes, as launchIteration: the
            // end nodes are never frozen (NF_DEFER), so they stay on the live
            // list and k_node_list rebuilds their conduit sums every
            // iteration; k_nc adds the non-conduit links in link order,
            // updates their depths and lists the unconverged ones for the next
            // walk (the walk skips LF_NC links: k_nc routes them)
            if (p.nNC > 0) hipLaunchKernelGGL(k_nc<false>, dim3(1), dim3(kBlock), 0, d->stream, p, k);
            if (multi)
                if (int r = flagExchange(d, k)) return r;
        }
        if (!p.qualUnfreeze)
            launchTimed(d, k_unfreeze, dim3(d->gridN), (hipEvent_t) nullptr, (hipEvent_t) nullptr, p);
    } else {
        for (int k = 0; k < p.maxTrials; k++)
            if (int r = launchIteration(d, k)) return r;
    }
    if (p.P > 0) {                                 // the link part runs in k_step_end
        if (multi)                                 // ghost links' concentrations (previous step end)
            if (int r = qualExchange(d)) return r;
        if (!d->fuseQual)
            launchTimed(d, k_qual_node, dim3(d->gridQ), ev ? ev[base] : nullptr, ev ? ev[base + 1] : nullptr, p);
    }
    launchTimed(d, stepEndKernel(d->fastLinks, d->allShapes, d->fuseQual), dim3(d->gridEnd),
                ev ? ev[base + 2] : nullptr, (hipEvent_t) nullptr, p);
    if (multi && (p.varStep || p.skipSteady)) {
        hipLaunchKernelGGL(k_finalize<1>, dim3(1), dim3(kBlock), 0, d->stream, p);
        if (p.varStep)                             // global Courant limits (min over ranks)
            if (int r = exchange(d, &p.ctl->stepRed[5], &p.ctl->stepRed[5], 2, 1)) return r;
        if (p.skipSteady)                          // the step's system flow totals (sum over ranks)
            if (int r = exchange(d, &p.ctl->steadyIO[0], &p.ctl->steadyIO[0], 6, 0)) return r;
        launchTimed(d, k_finalize<2>, dim3(1), (hipEvent_t) nullptr, ev ? ev[base + 3] : nullptr, p);
    } else {
        launchTimed(d, k_finalize<0>, dim3(1), (hipEvent_t) nullptr, ev ? ev[base + 3] : nullptr, p);
    }
    return 0;
}

// Start-up exchanges over the bootstrap: the host callback when one is set,
// else the RCCL communicator (n doubles, op 0 sum / 1 min, in place)
static int bootReduce(Router::Impl* d, double* buf, long n, int op)
{
    if (d->part.xchg) return hostReduce(d, buf, n, op);
    if (!d->comm) return xfail(d, "no bootstrap (host callback or RCCL communicator)");
    double* tmp = nullptr;
    if (hipMalloc(&tmp, n * sizeof(double)) != hipSuccess) return xfail(d, "bootstrap: hipMalloc");
    hipError_t e = hipMemcpy(tmp, buf, n * sizeof(double), hipMemcpyHostToDevice);
    ncclResult_t r = ncclSuccess;
    if (e == hipSuccess) r = ncclAllReduce(tmp, tmp, n, ncclDouble, op ? ncclMin : ncclSum, d->comm, d->stream);
    if (e == hipSuccess && r == ncclSuccess) {
        if (int w = waitDone(d, nullptr)) { (void)hipFree(tmp); return w; }
        e = hipMemcpy(buf, tmp, n * sizeof(double), hipMemcpyDeviceToHost);
    }
    (void)hipFree(tmp);
    if (r != ncclSuccess) return xfail(d, std::string("bootstrap ncclAllReduce: ") + ncclGetErrorString(r));
    if (e != hipSuccess) return xfail(d, std::string("bootstrap copy: ") + hipGetErrorString(e));
    return 0;
}

// XCHG_IPC start-up (Router::init, every rank): allocate this rank's uncached
// exchange region -- flag slots, reduction slots and the abort word at fixed
// offsets, then the ghost and concentration areas -- and all-gather over the
// bootstrap {its IPC handle, its ghost count, where each sender's ghosts start
// in it}; map every other rank's region (hipIpcOpenMemHandle), derive each
// send entry's slot in its receiver's area, and run one handshake flag
// exchange with a 10 s deadline.  Every rank reaches every bootstrap call
// whatever fails locally.  Returns 0 when the transport works on every rank,
// 1 when it does not (the caller falls back), 500 on a bootstrap error.
static int setupIpc(Router::Impl* d)
{
    Params& p = d->p;
    const Partition& part = d->part;
    const int R = part.nranks, me = part.rank;
    if (R > 64) return xfail(d, "the IPC transport takes at most 64 ranks");
    const size_t F = p.xF, P = p.P, nG = p.nGhost;
    const size_t flagW = 2 * (size_t)R, redW = 2 * (size_t)R * 2 * kRedMax, fixedW = flagW + redW + 8;
    const size_t words = fixedW + 2 * 2 * F * nG + 2 * 2 * P * nG;
    bool ok = hipExtMallocWithFlags(&d->ipcBase, words * 8, hipDeviceMallocUncached) == hipSuccess &&
              hipMemset(d->ipcBase, 0, words * 8) == hipSuccess;
    hipIpcMemHandle_t h{};
    ok = ok && hipIpcGetMemHandle(&h, d->ipcBase) == hipSuccess;
    (void)hipGetLastError();
    // record per rank: 64 handle bytes, ok, nGhost, its GPU's PCI address,
    // then per sender rank the start of its ghosts here + 1 (0: none) and
    // their count
    const int RH = 67, RL = RH + 2 * R;
    std::vector<double> rec((size_t)R * RL, 0.0);
    double* mine = rec.data() + (size_t)me * RL;
    const unsigned char* hb = (const unsigned char*)&h;
    static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle size");
    for (size_t i = 0; i < sizeof h; i++) mine[i] = hb[i];
    mine[64] = ok ? 1.0 : 0.0;
    mine[65] = (double)nG;
    {
        int dom = 0, bus = 0, dev = 0, ord = 0;
        (void)hipGetDevice(&ord);
        (void)hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, ord);
        (void)hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, ord);
        (void)hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, ord);
        (void)hipGetLastError();
        mine[66] = 1.0 + (double)dom * 65536.0 + (double)bus * 256.0 + (double)dev;
    }
    for (size_t k = 0; k < part.nbr.size(); k++) {
        mine[RH + 2 * part.nbr[k]] = part.recvOff[k] + 1.0;
        mine[RH + 1 + 2 * part.nbr[k]] = part.recvOff[k + 1] - part.recvOff[k];
    }
    if (int r = bootReduce(d, rec.data(), (long)rec.size(), 0)) return r;
    for (int r = 0; r < R; r++) ok = ok && rec[(size_t)r * RL + 64] == 1.0;
    {
        // every rank on a GPU of its own: the one-launch exchange
        std::vector<double> key(R);
        for (int r = 0; r < R; r++) key[r] = rec[(size_t)r * RL + 66];
        std::sort(key.begin(), key.end());
        const bool distinct = std::adjacent_find(key.begin(), key.end()) == key.end();
        d->xchgFused = d->xchgFusedEnv >= 0 ? d->xchgFusedEnv == 1 : distinct;
    }
    // map the peers' regions
    d->ipcPeer.assign(R, nullptr);
    std::vector<unsigned long long*> base(R, nullptr);
    base[me] = (unsigned long long*)d->ipcBase;
    for (int r = 0; r < R && ok; r++) {
        if (r == me) continue;
        hipIpcMemHandle_t hr{};
        unsigned char* b = (unsigned char*)&hr;
        for (size_t i = 0; i < sizeof hr; i++) b[i] = (unsigned char)rec[(size_t)r * RL + i];
        void* ptr = nullptr;
        if (hipIpcOpenMemHandle(&ptr, hr, hipIpcMemLazyEnablePeerAccess) != hipSuccess || !ptr) {
            (void)hipGetLastError();
            ok = false;
            break;
        }
        d->ipcPeer[r] = ptr;
        base[r] = (unsigned long long*)ptr;
    }
    // each send entry's receiver slot; every receiver expects exactly what is sent
    std::vector<int> sendNbr(std::max<size_t>(part.sendLink.size(), 1), 0), sendGi(sendNbr.size(), 0);
    std::vector<XPeer> xp(std::max<size_t>(part.nbr.size(), 1));
    for (size_t k = 0; k < part.nbr.size() && ok; k++) {
        const int r = part.nbr[k];
        const double* rr = rec.data() + (size_t)r * RL;
        const int ns = part.sendOff[k + 1] - part.sendOff[k];
        if (ns > 0 && (rr[RH + 2 * me] < 1.0 || (int)rr[RH + 1 + 2 * me] != ns)) { ok = false; break; }
        const int start = ns > 0 ? (int)rr[RH + 2 * me] - 1 : 0;
        const size_t ngr = (size_t)rr[65];
        xp[k].nGhost = (int)ngr;
        xp[k].ghost = base[r] + fixedW;
        xp[k].qual = base[r] + fixedW + 2 * 2 * F * ngr;
        for (int e = part.sendOff[k]; e < part.sendOff[k + 1]; e++) {
            sendNbr[e] = (int)k;
            sendGi[e] = start + (e - part.sendOff[k]);
        }
    }
    std::vector<int> ghostFrom(std::max<size_t>(nG, 1), -1);
    for (size_t k = 0; k < part.nbr.size(); k++)
        for (int g = part.recvOff[k]; g < part.recvOff[k + 1]; g++) ghostFrom[g] = part.nbr[k];
    {
        double a = ok ? 1.0 : 0.0;                 // every rank mapped every peer
        if (int r = bootReduce(d, &a, 1, 1)) return r;
        ok = a == 1.0;
    }
    if (!ok) return 1;
    // device tables
    std::vector<unsigned long long*> pf(R), pr(R), pa(R);
    for (int r = 0; r < R; r++) {
        pf[r] = base[r];
        pr[r] = base[r] + flagW;
        pa[r] = base[r] + flagW + redW;
    }
    auto up = [&](const void* src, size_t bytes) -> void* {
        void* q = nullptr;
        if (hipMalloc(&q, std::max<size_t>(bytes, 8)) != hipSuccess) return nullptr;
        d->allocs.push_back(q);
        if (!src) return hipMemset(q, 0, std::max<size_t>(bytes, 8)) == hipSuccess ? q : nullptr;
        if (bytes && hipMemcpy(q, src, bytes, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        return q;
    };
    p.xpeer = (const XPeer*)up(xp.data(), xp.size() * sizeof(XPeer));
    p.sendNbr = (const int*)up(sendNbr.data(), sendNbr.size() * sizeof(int));
    p.sendGi = (const int*)up(sendGi.data(), sendGi.size() * sizeof(int));
    p.ghostFrom = (const int*)up(ghostFrom.data(), ghostFrom.size() * sizeof(int));
    p.peerFlag = (unsigned long long* const*)up(pf.data(), R * sizeof(void*));
    p.peerRed = (unsigned long long* const*)up(pr.data(), R * sizeof(void*));
    p.peerAbort = (unsigned long long* const*)up(pa.data(), R * sizeof(void*));
    XCtl x0{};
    p.xctl = (XCtl*)up(&x0, sizeof x0);
    if (!p.xpeer || !p.sendNbr || !p.sendGi || !p.ghostFrom || !p.peerFlag || !p.peerRed || !p.peerAbort || !p.xctl)
        return xfail(d, "IPC transport: device tables");
    unsigned long long* own = base[me];
    p.flagRx = own;
    p.redRx = own + flagW;
    p.abortW = own + flagW + redW;
    p.ghostRx = own + fixedW;
    p.qualRx = own + fixedW + 2 * 2 * F * nG;
    p.xRank = me;
    p.xRanks = R;
    p.ipc = 1;
    // handshake: flag exchange number 1, every rank's flag set, 10 s at most
    int* dOk = (int*)up(nullptr, sizeof(int));
    if (!dOk) return xfail(d, "IPC transport: device tables");
    const long long tmo = p.xTimeout;
    p.xTimeout = std::min<long long>(tmo, (long long)(10.0 * d->wallKHz * 1000.0));
    hipLaunchKernelGGL(k_ipc_flag<true>, dim3(1), dim3(64), 0, d->stream, p, 0, dOk);
    p.xTimeout = tmo;
    int hv = 0;
    ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(d->stream) == hipSuccess &&
         hipMemcpy(&hv, dOk, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess && hv == 1 &&
         d->xerrHost[0] == 0;
    {
        double a = ok ? 1.0 : 0.0;
        if (int r = bootReduce(d, &a, 1, 1)) return r;
        ok = a == 1.0;
    }
    if (!ok) {
        p.ipc = 0;
        return 1;
    }
    return 0;
}

int Router::init(Project& prj, int device, const Partition* partIn)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    Network& net = prj.net;
    State& st = prj.st;
    int nN = net.nNodes(), nL = net.nLinks(), P = prj.opt.ignoreQuality ? 0 : net.nPollut();
    // local view: the whole network on one GPU, or this rank's part of it
    if (partIn) d->part = *partIn;
    else d->part.nranks = 1;
    {
        std::string m;
        if (buildPartition(net, d->part, &m)) { fail(m); return err_; }
    }
    const Partition& part = d->part;
    // local links: this rank's owned links, then its ghost links (other
    // ranks' links touching a held node; values received every iteration)
    std::vector<int> LL = part.llink;
    LL.insert(LL.end(), part.lghost.begin(), part.lghost.end());
    const std::vector<int>& LN = part.lnode;
    const int nOwn = (int)part.llink.size();
    nN = (int)LN.size();
    nL = (int)LL.size();
    auto gl = [&](const std::vector<double>& v) {
        std::vector<double> o(nL);
        for (int j = 0; j < nL; j++) o[j] = v[LL[j]];
        return o;
    };
    auto gn = [&](const std::vector<double>& v) {
        std::vector<double> o(nN);
        for (int i = 0; i < nN; i++) o[i] = v[LN[i]];
        return o;
    };
    auto gni = [&](const std::vector<int>& v) {
        std::vector<int> o(nN);
        for (int i = 0; i < nN; i++) o[i] = v[LN[i]];
        return o;
    };
    auto gq = [&](const std::vector<double>& v, int nObj, const std::vector<int>& map) {
        std::vector<double> o((size_t)P * map.size());
        for (int q = 0; q < P; q++)
            for (size_t k = 0; k < map.size(); k++) o[(size_t)q * map.size() + k] = v[(size_t)q * nObj + map[k]];
        return o;
    };
    const int gN = net.nNodes(), gL = net.nLinks();
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        fail("no HIP device available (the MI355X engine has no CPU fallback)");
        return err_;
    }
    if (device < 0 || device >= ndev) device = 0;
    HIPCHECK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPCHECK(hipGetDeviceProperties(&prop, device));
    {
        int wr = 0;                                // wall_clock64 rate (kHz), for the phase probe
        if (hipDeviceGetAttribute(&wr, hipDeviceAttributeWallClockRate, device) == hipSuccess && wr > 0)
            d->wallKHz = wr;
    }
    devName_ = std::string("hip:") + prop.gcnArchName + ":" + prop.name;
    HIPCHECK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    HIPCHECK(hipStreamCreateWithFlags(&d->side, hipStreamNonBlocking));
    {
        const int m = std::max(prj.opt.maxTrials, 1);
        d->forkEv.assign(m, nullptr);
        d->joinEv.assign(m, nullptr);
        for (int k = 0; k < m; k++) {
            HIPCHECK(hipEventCreateWithFlags(&d->forkEv[k], hipEventDisableTiming));
            HIPCHECK(hipEventCreateWithFlags(&d->joinEv[k], hipEventDisableTiming));
        }
    }

    Params& p = d->p;
    p.nN = nN; p.nL = nOwn; p.nLs = nL; p.P = P;
    p.maxTrials = prj.opt.maxTrials;
    p.surchargeMethod = prj.opt.surchargeMethod;
    p.forceMainEqn = prj.opt.forceMainEqn;
    p.inertDamping = prj.opt.inertDamping;
    p.normalFlowLtd = prj.opt.normalFlowLtd;
    p.allowPonding = prj.opt.allowPonding;
    p.crownCutoff = prj.opt.crownCutoff;
    p.minSurfArea = prj.opt.minSurfArea;
    p.headTol = prj.opt.headTol;
    p.courantFactor = prj.opt.courantFactor;
    p.minRouteStep = prj.opt.minRouteStep;
    p.routeStep = prj.opt.routeStep;
    p.varStep = (prj.opt.courantFactor != 0.0 && prj.opt.routeStep >= 0.001) ? 1 : 0;
    // SKIP_STEADY_STATE (routing.c:236-244, 383-395); with several ranks the
    // inflow test and the step's flow totals are reduced over the ranks once
    // per step each (launchStep), so every rank makes the same decision
    p.skipSteady = prj.opt.skipSteadyState ? 1 : 0;
    p.sysFlowTol = prj.opt.sysFlowTol;
    p.latFlowTol = prj.opt.latFlowTol;

    hipError_t e;
    auto upD = [&](const std::vector<double>& v, size_t n) -> double* {
        double* ptr = devAlloc<double>(d, n, &e);
        if (e == hipSuccess && n) e = hipMemcpy(ptr, v.data(), n * sizeof(double), hipMemcpyHostToDevice);
        return ptr;
    };
    auto upI = [&](const std::vector<int>& v, size_t n) -> int* {
        int* ptr = devAlloc<int>(d, n, &e);
        if (e == hipSuccess && n) e = hipMemcpy(ptr, v.data(), n * sizeof(int), hipMemcpyHostToDevice);
        return ptr;
    };
#define UPD(dst, vec, n) do { dst = upD(vec, n); if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; } } while (0)
#define UPI(dst, vec, n) do { dst = upI(vec, n); if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; } } while (0)

    // ---- link static ------------------------------------------------------
    std::vector<int> nodes2((size_t)nL * 2);
    std::vector<int> lflags(nL), coldLinks, outLinks;
    std::vector<double> inv1(nL), inv2(nL), xd[11];
    for (auto& v : xd) v.resize(nL);
    for (int j = 0; j < nL; j++) {
        const int g = LL[j];                        // global link index
        int n1 = net.node1[g], n2 = net.node2[g];   // global node indices
        nodes2[2 * j] = part.gnode[n1];
        nodes2[2 * j + 1] = part.gnode[n2];
        inv1[j] = net.invertElev[n1];
        inv2[j] = net.invertElev[n2];
        const Xsect& x = net.xsect[g];
        uint32_t f = (uint32_t)x.type & LF_XTYPE;
        f |= ((uint32_t)net.barrels[g] & 0xFFu) << LF_BARREL_SHIFT;
        if (net.hasLosses[g]) f |= LF_LOSSES;
        if (net.hasFlapGate[g]) f |= LF_FLAP;
        if (net.nodeType[n1] == OUTFALL) { f |= LF_N1_OUTFALL; if (net.outfallFlap[n1]) f |= LF_N1_OFLAP; }
        if (net.nodeType[n2] == OUTFALL) { f |= LF_N2_OUTFALL; if (net.outfallFlap[n2]) f |= LF_N2_OFLAP; }
        if (net.seepRate[g] > 0.0 || (prj.evapCanBePositive() && isOpen(x.type))) f |= LF_SEEP;
        if (net.qLimit[g] > 0.0) f |= LF_QLIMIT;
        if (net.direction[g] < 0) f |= LF_DIRNEG;
        if (j >= nOwn) {
            f |= LF_COLD;                           // ghost: computed by its owner, never here
        } else if (!net.isTrueConduit(g)) {
            f |= LF_NC | LF_COLD;                   // k_nc, not the conduit kernels
            if (net.linkType[g] == PUMP) f |= LF_PUMP;
            if (net.linkType[g] == CONDUIT) f |= LF_DUMMY;
        } else if (net.offset1[g] > 0.0 || net.offset2[g] > 0.0 || !isBasicShape(x.type) ||
                   x.culvertCode > 0) {
            if (x.culvertCode > 0) f |= ((uint32_t)std::min(x.culvertCode, 63) & 0x3Fu) << LF_CULVERT_SHIFT;
            f |= LF_COLD;
            coldLinks.push_back(j);
        }
        lflags[j] = (int)f;
        xd[0][j] = x.yFull; xd[1][j] = x.wMax; xd[2][j] = x.ywMax; xd[3][j] = x.aFull;
        xd[4][j] = x.rFull; xd[5][j] = x.sFull; xd[6][j] = x.sMax; xd[7][j] = x.yBot;
        xd[8][j] = x.aBot; xd[9][j] = x.sBot; xd[10][j] = x.rBot;
    }
    // kFast: every streaming conduit circular, no SLOT surcharge, and at most
    // kGeomMax distinct sections; the sections become one LDS table and each
    // streaming conduit's flags carry its section id
    std::vector<double> geomTab;
    {
        bool fast = prj.opt.surchargeMethod != SUR_SLOT;
        const char* gl = getenv("SWMM5_GENERIC_LINKS");
        if (gl && atoi(gl)) fast = false;
        std::map<std::array<double, 7>, int> ids;
        std::vector<int> gid(nL, 0);
        for (int j = 0; j < nL && fast; j++) {
            if (lflags[j] & LF_COLD) continue;
            if ((lflags[j] & LF_XTYPE) != G_CIRCULAR) { fast = false; break; }
            std::array<double, 7> key = {xd[0][j], xd[1][j], xd[3][j], xd[4][j], xd[5][j], xd[6][j], xd[2][j]};
            auto it = ids.find(key);
            if (it == ids.end()) {
                if ((int)ids.size() == kGeomMax) { fast = false; break; }
                it = ids.emplace(key, (int)ids.size()).first;
                geomTab.insert(geomTab.end(), key.begin(), key.end());
                double rh, rl;
                recipDD(key[0], &rh, &rl);
                geomTab.push_back(rh);
                geomTab.push_back(rl);
            }
            gid[j] = it->second;
        }
        d->fastLinks = fast;
        p.nGeom = fast ? (int)ids.size() : 0;
        if (fast)
            for (int j = 0; j < nL; j++)
                if (!(lflags[j] & LF_COLD))
                    lflags[j] = (int)((uint32_t)lflags[j] | ((uint32_t)gid[j] << LF_GEOM_SHIFT));
        if (!fast) geomTab.clear();
    }
    {
        int* ptr = upI(nodes2, nodes2.size());
        if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
        p.lnodes = (const int2*)ptr;
        int* fl;
        UPI(fl, lflags, nL);
        p.lflags = (const uint32_t*)fl;
        int* cl;
        UPI(cl, coldLinks, coldLinks.size());
        p.coldLinks = cl;
        p.nCold = (int)coldLinks.size();

    }
    double* tmp;
    UPD(tmp, inv1, nL); p.inv1 = tmp;
    UPD(tmp, inv2, nL); p.inv2 = tmp;
    UPD(tmp, gl(net.offset1), nL); p.off1 = tmp;
    UPD(tmp, gl(net.offset2), nL); p.off2 = tmp;
    UPD(tmp, xd[0], nL); p.yFull = tmp;
    UPD(tmp, xd[1], nL); p.wMax = tmp;
    UPD(tmp, xd[2], nL); p.ywMax = tmp;
    UPD(tmp, xd[3], nL); p.aFull = tmp;
    UPD(tmp, xd[4], nL); p.rFull = tmp;
    UPD(tmp, xd[5], nL); p.sFull = tmp;
    UPD(tmp, xd[6], nL); p.sMax = tmp;
    UPD(tmp, xd[7], nL); p.yBot = tmp;
    UPD(tmp, xd[8], nL); p.aBot = tmp;
    UPD(tmp, xd[9], nL); p.sBot = tmp;
    UPD(tmp, xd[10], nL); p.rBot = tmp;
    UPD(tmp, gl(net.lengthT), nL); p.length = tmp;
    p.lengthRaw = p.length;
    if (net.length != net.lengthT) { UPD(tmp, gl(net.length), nL); p.lengthRaw = tmp; }
    UPD(tmp, gl(net.modLength), nL); p.modLength = tmp;
    UPD(tmp, gl(net.roughFactor), nL); p.roughFactor = tmp;
    UPD(tmp, gl(net.beta), nL); p.beta = tmp;
    UPD(tmp, gl(net.qMax), nL); p.qMax = tmp;
    UPD(tmp, gl(net.qLimit), nL); p.qLimit = tmp;
    UPD(tmp, gl(net.slope), nL); p.slope = tmp;
    UPD(tmp, gl(net.cLossInlet), nL); p.cIn = tmp;
    UPD(tmp, gl(net.cLossOutlet), nL); p.cOut = tmp;
    UPD(tmp, gl(net.cLossAvg), nL); p.cAvg = tmp;
    UPD(tmp, gl(net.seepRate), nL); p.seepRate = tmp;
    // ---- link dynamic -----------------------------------------------------
    UPD(p.lNewFlow, gl(st.lNewFlow), nL);
    UPD(p.lOldFlow, gl(st.lOldFlow), nL);
    UPD(p.lNewDepth, gl(st.lNewDepth), nL);
    UPD(p.lOldDepth, gl(st.lOldDepth), nL);
    UPD(p.lNewVolume, gl(st.lNewVolume), nL);
    UPD(p.lOldVolume, gl(st.lOldVolume), nL);
    UPD(p.a1, gl(st.a1), nL);
    UPD(p.a2, gl(st.a2), nL);
    UPD(p.q1, gl(st.q1), nL);
    UPD(p.dqdh, gl(st.dqdh), nL);
    UPD(p.froude, gl(st.froude), nL);
    UPD(p.sa1, gl(st.surfArea1), nL);
    UPD(p.sa2, gl(st.surfArea2), nL);
    UPD(p.evapLoss, gl(st.evapLossRate), nL);
    UPD(p.seepLoss, gl(st.seepLossRate), nL);
    UPD(p.setting, gl(st.setting), nL);
    {                                              // Params::rare
        const RareLink rl{p.cIn, p.cOut, p.cAvg, p.qLimit, p.evapLoss, p.seepLoss};
        RareLink* dr = devAlloc<RareLink>(d, 1, &e);
        if (e == hipSuccess) e = hipMemcpy(dr, &rl, sizeof(RareLink), hipMemcpyHostToDevice);
        if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
        p.rare = dr;
    }
    {
        std::vector<int> ls(nL);
        for (int j = 0; j < nL; j++) {
            const int g = LL[j];
            ls[j] = st.flowClass[g] | (st.fullState[g] << 4) | (st.normalFlow[g] << 8) |
                    (st.capacityLimited[g] << 9);
        }
        UPI(p.lstate, ls, nL);
    }
    // ---- node static ------------------------------------------------------
    std::vector<int> nflags(nN), outLink(nN, -1);
    std::vector<double> yCrown(nN);
    for (int i = 0; i < nN; i++) {
        const int g = LN[i];                        // global node index
        uint32_t f = (uint32_t)net.nodeType[g] & NF_TYPE;
        if (net.nodeType[g] == OUTFALL) f |= ((uint32_t)net.outfallType[g] & 0x7u) << NF_OTYPE_SHIFT;
        if (net.degree[g] < 0) f |= NF_DEGNEG;
        if (prj.opt.allowPonding && net.pondedArea[g] > 0.0) f |= NF_CANPOND;
        if (net.degree[g] == 0) f |= NF_DEG0;
        if (part.hasGhost[i]) f |= NF_SHARED;      // sums include received ghost values
        if (!part.owned[i]) f |= NF_REPLICA;
        nflags[i] = (int)f;
        yCrown[i] = net.crownElev[g] - net.invertElev[g];
    }
    // tidal-curve / stage-time-series outfalls: their (x, y) tables
    p.ofTab = nullptr;
    p.ofOff = nullptr;
    {
        std::vector<double> tab;
        std::vector<int> off(2 * nN, -1);
        for (int i = 0; i < nN; i++) {
            const int g = LN[i];
            if (net.nodeType[g] != OUTFALL || net.outfallType[g] <= O_FIXED) continue;
            const std::vector<double>* xs;
            const std::vector<double>* ys;
            if (net.outfallType[g] == O_TIDAL) { xs = &net.curves[net.outfallSeries[g]].x; ys = &net.curves[net.outfallSeries[g]].y; }
            else { xs = &net.tseries[net.outfallSeries[g]].x; ys = &net.tseries[net.outfallSeries[g]].y; }
            off[2 * i] = (int)tab.size();
            off[2 * i + 1] = (int)xs->size();
            for (size_t m = 0; m < xs->size(); m++) { tab.push_back((*xs)[m]); tab.push_back((*ys)[m]); }
        }
        if (!tab.empty()) {
            UPD(tmp, tab, tab.size()); p.ofTab = tmp;
            int* o;
            UPI(o, off, off.size());
            p.ofOff = o;
        }
    }
    p.startDateTime = prj.opt.startDateTime;
    // CSR: incident links per node, ascending link index (all links are true
    // conduits, so this is exactly the order of dynwave.c:398-401)
    // Pumps / regulators are not in it: their flows join the node sums after
    // all conduits (dynwave.c:398-412), in k_nc.  The quality CSR keeps every
    // link in link order (findLinkMassFlow, qualrout.c:111).
    std::vector<int> rowptr, csr, qrowptr, qcsr;
    buildLocalCsr(net, part, true, rowptr, csr);
    bool anyNC = false;                             // pumps, regulators or DUMMY conduits
    for (int g = 0; g < gL && !anyNC; g++) anyNC = !net.isTrueConduit(g);
    if (anyNC) buildLocalCsr(net, part, false, qrowptr, qcsr);
    // the reference's link_setOutfallDepth loop (findNodeDepths): the last
    // link touching an outfall sets its depth
    for (int j = 0; j < nOwn; j++) {
        int a = nodes2[2 * j], b = nodes2[2 * j + 1];
        if (net.nodeType[LN[b]] == OUTFALL) outLink[b] = j;
        else if (net.nodeType[LN[a]] == OUTFALL) outLink[a] = j;
    }
    for (int i = 0; i < nN; i++)
        if (outLink[i] >= 0) outLinks.push_back(outLink[i]);
    std::sort(outLinks.begin(), outLinks.end());
    {
        int* cl;
        UPI(cl, outLinks, outLinks.size());
        p.outLinks = cl;
        int* inl[4] = {&p.outInl0, &p.outInl1, &p.outInl2, &p.outInl3};
        for (int c = 0; c < 4; c++) *inl[c] = (c < (int)outLinks.size()) ? outLinks[c] : -1;
        std::vector<int> on(outLinks.size());
        for (size_t c = 0; c < outLinks.size(); c++) {
            const int j = outLinks[c];
            on[c] = ((uint32_t)lflags[j] & LF_N2_OUTFALL) ? nodes2[2 * j + 1] : nodes2[2 * j];
        }
        int* onp;
        UPI(onp, on, on.size());
        p.outNodes = onp;
        int* ond[4] = {&p.outNd0, &p.outNd1, &p.outNd2, &p.outNd3};
        for (int c = 0; c < 4; c++) *ond[c] = (c < (int)on.size()) ? on[c] : -1;
        p.nOutLinks = getenv("SWMM5_TIMING_NO_OUTFALL") ? 0 : (int)outLinks.size();   // timing experiment only
    }
    // deferred outfall depths (k_walk, deferredOutfalls): every conduit with an
    // outfall end is its outfall's only link, listed in outLinks, has one
    // outfall end and streams (not cold, not a pump / regulator / DUMMY)
    bool outfallsDeferrable = p.nOutLinks >= 1 && p.nOutLinks <= 64;
    {
        int withOutfall = 0;
        for (int j = 0; j < nOwn && outfallsDeferrable; j++) {
            const uint32_t f = (uint32_t)lflags[j];
            const bool o1 = (f & LF_N1_OUTFALL) != 0, o2 = (f & LF_N2_OUTFALL) != 0;
            if (!o1 && !o2) continue;
            withOutfall++;
            if ((o1 && o2) || (f & (LF_COLD | LF_NC))) outfallsDeferrable = false;
        }
        if (withOutfall != p.nOutLinks) outfallsDeferrable = false;
    }
    // end nodes of pumps / regulators: depth updated by k_nc
    std::vector<int> defNodes;
    {
        std::vector<char> isDef(nN, 0);
        for (int j = 0; j < nOwn; j++)
            if (lflags[j] & LF_NC) { isDef[nodes2[2 * j]] = 1; isDef[nodes2[2 * j + 1]] = 1; }
        for (int i = 0; i < nN; i++)
            if (isDef[i]) { defNodes.push_back(i); nflags[i] = (int)((uint32_t)nflags[i] | NF_DEFER); }
    }
    d->nE = (int)csr.size();
    {
        int* fl;
        UPI(fl, nflags, nN);
        p.nflags = (const uint32_t*)fl;
        int* rp;
        UPI(rp, rowptr, nN + 1); p.rowptr = rp;
        UPI(rp, csr, csr.size()); p.csr = rp;
        {
            std::vector<int> other(csr.size(), -1);
            for (int i = 0; i < nN; i++)
                for (int e = rowptr[i]; e < rowptr[i + 1]; e++) {
                    const int l = csr[e] & 0x7FFFFFFF;
                    other[e] = (csr[e] < 0) ? nodes2[2 * l] : nodes2[2 * l + 1];
                }
            UPI(rp, other, other.size()); p.csrOther = rp;
        }
        if (anyNC) {
            UPI(rp, qrowptr, nN + 1); p.qrowptr = rp;
            UPI(rp, qcsr, qcsr.size()); p.qcsr = rp;
        } else {
            p.qrowptr = p.rowptr;
            p.qcsr = p.csr;
        }
        p.nDef = (int)defNodes.size();
        UPI(rp, defNodes, defNodes.size()); p.defNodes = rp;
        UPI(rp, outLink, nN); p.outfallLink = rp;
    }
    UPD(tmp, gn(net.invertElev), nN); p.invert = tmp;
    UPD(tmp, gn(net.fullDepth), nN); p.fullDepth = tmp;
    UPD(tmp, gn(net.surDepth), nN); p.surDepth = tmp;
    UPD(tmp, gn(net.pondedArea), nN); p.pondedArea = tmp;
    UPD(tmp, yCrown, nN); p.yCrown = tmp;
    UPD(tmp, gn(net.crownElev), nN); p.crownElev = tmp;
    UPD(tmp, gn(net.fullVolume), nN); p.fullVolume = tmp;
    UPD(tmp, gn(net.fixedStage), nN); p.fixedStage = tmp;
    // ---- storage units -------------------------------------------------------
    {
        std::vector<int> shape(nN, -1), coff(nN, 0), cn(nN, 0);
        std::vector<double> cx, cy;
        std::vector<int> curveOff(net.curves.size(), 0);   // every curve, in one table
        for (size_t c = 0; c < net.curves.size(); c++) {
            curveOff[c] = (int)cx.size();
            cx.insert(cx.end(), net.curves[c].x.begin(), net.curves[c].x.end());
            cy.insert(cy.end(), net.curves[c].y.begin(), net.curves[c].y.end());
        }
        for (int i = 0; i < nN; i++) {
            const int g = LN[i];
            if (net.nodeType[g] != STORAGE) continue;
            shape[i] = net.stShape[g];
            int c = net.stCurve[g];
            if (c >= 0) {
                coff[i] = curveOff[c];
                cn[i] = (int)net.curves[c].x.size();
            }
        }
        if (cx.empty()) { cx.push_back(0.0); cy.push_back(0.0); }
        int* ip;
        UPI(ip, shape, nN); p.stShape = ip;
        UPI(ip, coff, nN); p.stCOff = ip;
        UPI(ip, cn, nN); p.stCN = ip;
        UPD(tmp, gn(net.stA0), nN); p.stA0 = tmp;
        UPD(tmp, gn(net.stA1), nN); p.stA1 = tmp;
        UPD(tmp, gn(net.stA2), nN); p.stA2 = tmp;
        UPD(tmp, gn(net.stFEvap), nN); p.stFEvap = tmp;
        UPD(tmp, cx, cx.size()); p.curveX = tmp;
        UPD(tmp, cy, cy.size()); p.curveY = tmp;
        p.ucfL = prj.ucfLength();
        p.ucfV = prj.ucfVolume();
        // pumps / regulators (k_nc), link order
        {
            std::vector<int> ncl;
            std::vector<NcLink> ncs;
            std::vector<double> coef, target, zero;
            for (int j = 0; j < nOwn; j++) {
                const int g = LL[j];
                if (net.isTrueConduit(g)) continue;
                ncl.push_back(j);
                NcLink L = prj.ncLink(g);          // DUMMY conduits: type LK_CONDUIT
                int c = net.ncCurve[g];
                L.cOff = c >= 0 ? curveOff[c] : 0;
                ncs.push_back(L);
                coef.push_back(st.ncCOrif[g]);
                coef.push_back(st.ncCWeir[g]);
                coef.push_back(st.ncHCrit[g]);
                coef.push_back(st.ncCSurch[g]);
                target.push_back(st.targetSetting[g]);
                zero.push_back(0.0);
            }
            p.nNC = (int)ncl.size();
            if (ncl.empty()) { ncl.push_back(0); ncs.push_back(NcLink{}); coef.assign(4, 0.0); target.push_back(0.0); zero.push_back(0.0); }
            int* ip2;
            UPI(ip2, ncl, ncl.size()); p.ncLinks = ip2;
            NcLink* dl = devAlloc<NcLink>(d, ncs.size(), &e);
            if (e == hipSuccess) e = hipMemcpy(dl, ncs.data(), ncs.size() * sizeof(NcLink), hipMemcpyHostToDevice);
            if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
            p.ncL = dl;
            UPD(p.ncCoef, coef, coef.size());
            UPD(p.ncTarget, target, target.size());
            UPD(p.ncSurf, zero, zero.size());
            UPD(p.ncQ, zero, zero.size());
            std::vector<int> zi(zero.size(), 0);
            UPI(p.ncBypass, zi, zi.size());
            std::vector<double> zl(nL, 0.0);
            for (double** a : {&p.pUtil, &p.pAvg, &p.pVol, &p.pEnergy, &p.pOffLow, &p.pOffHigh, &p.pMin, &p.pMax})
                UPD(*a, zl, nL);
            std::vector<int> zil(nL, 0);
            UPI(p.pStarts, zil, nL);
            UPI(p.pPeriods, zil, nL);
        }
        std::vector<double> z(nN, 0.0);
        UPD(p.nPrevDepth, gn(st.newDepth), nN);
        UPD(p.nLosses, z, nN);
        UPD(p.nEvapVol, z, nN);
        UPD(p.nExfilVol, z, nN);
        {   // storage seepage objects (createStorageExfil + exfil_initState)
            std::vector<int> xi(nN, -1);
            std::vector<double> xd;
            for (int i = 0; i < nN; i++) {
                const int g = LN[i];
                if (net.nodeType[g] != STORAGE || net.stExKs[g] == 0.0) continue;
                xi[i] = (int)(xd.size() / kExVals);
                xd.resize(xd.size() + kExVals);
                exfilInit(prj.storageGeom(g), net.stExS[g], net.stExKs[g], net.stExIMD[g],
                          xd.data() + xd.size() - kExVals);
            }
            if (xd.empty()) xd.assign(kExVals, 0.0);
            int* ip3;
            UPI(ip3, xi, nN); p.exIdx = ip3;
            UPD(p.exData, xd, xd.size());
        }
        std::vector<double> h(nN, 0.0);
        if (!st.hrt.empty()) h = gn(st.hrt);
        UPD(p.hrt, h, nN);
    }
    // ---- node dynamic -----------------------------------------------------
    UPD(p.nNewDepth, gn(st.newDepth), nN);
    UPD(p.nOldDepth, gn(st.oldDepth), nN);
    UPD(p.nNewVolume, gn(st.newVolume), nN);
    UPD(p.nOldVolume, gn(st.oldVolume), nN);
    UPD(p.inflow, gn(st.inflow), nN);
    UPD(p.outflow, gn(st.outflow), nN);
    UPD(p.overflow, gn(st.overflow), nN);
    UPD(p.newLat, gn(st.newLatFlow), nN);
    UPD(p.oldLat, gn(st.oldLatFlow), nN);
    UPD(p.oldNetInflow, gn(st.oldNetInflow), nN);
    UPD(p.oldFlowInflow, gn(st.oldFlowInflow), nN);
    UPD(p.oldSurfArea, gn(st.oldSurfArea), nN);
    {   // gather-reuse sums (written by every gather before any reuse) and flags
        std::vector<double> zN(nN, 0.0);
        UPD(p.nSurf, zN, nN);
        UPD(p.nDqdh, zN, nN);
        UPD(p.yRaw, zN, nN);
        std::vector<double> ym(nN);
        for (size_t i = 0; i < nN; i++) ym[i] = net.fullDepth[LN[i]] + net.surDepth[LN[i]];
        UPD(p.yMaxNP, ym, nN);
        p.ulist = devAlloc<int>(d, 2 * (size_t)nN, &e);
        if (e == hipSuccess) p.ulistRow = devAlloc<int2>(d, 2 * (size_t)nN, &e);
        if (e == hipSuccess) p.vlist = devAlloc<int>(d, 2 * (size_t)nN, &e);
        if (e == hipSuccess) p.vlistRow = devAlloc<int2>(d, 2 * (size_t)nN, &e);
        if (e == hipSuccess) p.wlist = devAlloc<int>(d, (size_t)nN, &e);
        if (e == hipSuccess) p.wmark = devAlloc<int>(d, (size_t)nN, &e);
        if (e == hipSuccess) e = hipMemset(p.wmark, 0, std::max<size_t>(nN, 1) * sizeof(int));
        if (e == hipSuccess) p.nstamp = devAlloc<unsigned>(d, (size_t)nN, &e);
        if (e == hipSuccess) e = hipMemset(p.nstamp, 0xFF, std::max<size_t>(nN, 1) * sizeof(unsigned));
        if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
        p.dirty = devAlloc<unsigned char>(d, nN, &e);
        if (e == hipSuccess) e = hipMemset(p.dirty, 0, std::max<size_t>(nN, 1));
        if (e == hipSuccess) p.nodeWork = devAlloc<unsigned>(d, nN, &e);
        if (e == hipSuccess) e = hipMemset(p.nodeWork, 0, std::max<size_t>(nN, 1) * sizeof(unsigned));
        if (e == hipSuccess) p.nodeLinkWork = devAlloc<unsigned>(d, nN, &e);
        if (e == hipSuccess) e = hipMemset(p.nodeLinkWork, 0, std::max<size_t>(nN, 1) * sizeof(unsigned));
        if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
        p.frz = devAlloc<unsigned char>(d, nN, &e);
        if (e == hipSuccess) e = hipMemset(p.frz, 0, std::max<size_t>(nN, 1));
        if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
        // a frozen junction's later updates are pure relaxation steps whose
        // change halves each iteration (freezable); a tolerance below a few
        // ulps of a depth would not absorb their rounding.  SWMM5_NO_FREEZE
        // disables it (comparison runs)
        const char* nf = getenv("SWMM5_NO_FREEZE");
        p.freeze = (prj.opt.headTol > 1e-12 && p.maxTrials > 2 && !(nf && atoi(nf))) ? 1 : 0;
    }
    UPD(p.dYdT, gn(st.dYdT), nN);
    UPI(p.conv, gni(st.converged), nN);
    // ---- inflows ----------------------------------------------------------
    d->constantInflow = prj.inflowsAreConstant();
    {
        std::vector<double> lat, qual;
        double tot[3];
        prj.evalInflows(prj.getDateTime(0.0), lat, P ? &qual : nullptr, &tot[0], &tot[1], &tot[2]);
        // system inflow totals are counted once (rank 0); a node's own inflow
        // is added by its owner only (replicas start their sums from 0)
        if (part.rank != 0) tot[0] = tot[1] = tot[2] = 0.0;
        d->latTot0[0] = tot[0]; d->latTot0[1] = tot[1]; d->latTot0[2] = tot[2];
        std::vector<double> latL(nN);                   // every replica adds the node's own inflow
        for (int i = 0; i < nN; i++) latL[i] = lat[LN[i]];
        UPD(d->latBase, latL, nN);
        if (P) {
            UPD(d->qualBase, gq(qual, gN, LN), (size_t)P * nN);
        } else {
            d->qualBase = devAlloc<double>(d, 1, &e);
        }
    }
    p.latIn = d->latBase;
    p.qualIn = d->qualBase;
    // ---- quality ----------------------------------------------------------
    {
        std::vector<double> kd(std::max(P, 1), 0.0);
        for (int q = 0; q < P; q++) kd[q] = net.pollut[q].kDecay;
        UPD(tmp, kd, kd.size()); p.kDecay = tmp;
        size_t nq = (size_t)std::max(P, 0);
        // qualPar starts at 0: [0] holds the latest concentrations
        UPD(p.nQual[0], gq(st.nNewQual, gN, LN), nq * nN);
        UPD(p.nQual[1], gq(st.nOldQual, gN, LN), nq * nN);
        UPD(p.lQual[0], gq(st.lNewQual, gL, LL), nq * nL);
        UPD(p.lQual[1], gq(st.lOldQual, gL, LL), nq * nL);
    }
    // ---- tables, partials, control ---------------------------------------
    {
        std::vector<double> t(&SWX_CIRC_TABLES[0][0], &SWX_CIRC_TABLES[0][0] + 5 * SWX_CIRC_N);
        t.insert(t.end(), geomTab.begin(), geomTab.end());
        UPD(tmp, t, t.size()); p.gTables = tmp;
        std::vector<double> st(SWX_SHAPE_TAB, SWX_SHAPE_TAB + SWX_SHAPE_TAB_LEN);
        UPD(tmp, st, st.size()); p.gShapeTab = tmp;
        p.gXTab = nullptr;
        p.lTabOff = nullptr;
        if (!prj.net.xTab.empty()) {
            UPD(tmp, prj.net.xTab, prj.net.xTab.size()); p.gXTab = tmp;
            std::vector<int> off(nL, -1);
            for (int j = 0; j < nL; j++) off[j] = prj.net.xsect[LL[j]].tabOff;
            int* o;
            UPI(o, off, nL);
            p.lTabOff = o;
        }
    }
    if (const char* w = getenv("SWMM5_LINK_WAVES")) d->linkWaves = atoi(w);
    for (int j = 0; j < nL; j++)
        if (!isBasicShape((int)(lflags[j] & LF_XTYPE))) d->allShapes = true;
    d->general = prj.net.nStorage > 0 || d->allShapes;
    int maxBlocks = 8 * std::max(prop.multiProcessorCount, 1);
    // streaming kernels: one resident wave of workgroups (grid-stride loops),
    // so early-exited Picard iterations dispatch few workgroups
    auto resident = [&](const void* fn, int n, double factor = 1.0) {
        int per = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, kBlock, 0) != hipSuccess || per < 1)
            per = 2;
        int cap = (int)(per * std::max(prop.multiProcessorCount, 1) * factor);
        if (const char* g = getenv("SWMM5_GRID_FACTOR")) cap = (int)(cap * atof(g));
        return std::max(1, std::min((n + kBlock - 1) / kBlock, std::max(cap, 1)));
    };
    d->gridL = resident((const void*)linkKernel(false, d->linkWaves, d->fastLinks), nL);
    // k_node: one resident wave of workgroups (round 4, q = 0.12 regime:
    // k_node(1) 34.8 -> 31.8 us against two waves, which round 3's lighter
    // regime preferred); the quality kernel keeps two (gridQ: 62 against
    // 71 us with one)
    double nodeFactor = 1.0;
    if (const char* g = getenv("SWMM5_NODE_GRID_FACTOR")) nodeFactor = atof(g);
    d->gridN = resident((const void*)nodeKernel(false, d->general), nN, nodeFactor);
    d->gridQ = resident((const void*)nodeKernel(false, d->general), nN, 2.0);
    // iterations k >= 2 walk the unconverged list (four threads per node):
    // two workgroups per CU (round 4: ≈15,000-20,000 listed nodes, walk
    // 17.4 -> 13.8 us eager, 0.4643 -> 0.4471 ms/step with the node grid
    // above; one per CU was best for round 3's few thousand)
    d->gridLinkSparse = std::max(1, std::min(d->gridL, 2 * std::max(prop.multiProcessorCount, 1)));
    if (const char* g = getenv("SWMM5_LINK_SPARSE_GRID_FACTOR"))
        d->gridLinkSparse = std::max(1, std::min(d->gridL, (int)(atof(g) * std::max(prop.multiProcessorCount, 1))));
    d->gridC = std::max(1, std::min((p.nCold + kBlock - 1) / kBlock, maxBlocks));
    // list graph node kernel: two workgroups per CU (the live lists are tens
    // of thousands of nodes at most in its range)
    {
        double f = 2.0;
        if (const char* g = getenv("SWMM5_NODE_LIST_GRID")) f = atof(g);
        d->gridNList = std::max(1, (int)(f * std::max(prop.multiProcessorCount, 1)));
    }
    // quality fused into the step end (k_step_end<..., kQual>) only with
    // SWMM5_FUSE_QUAL=1: bitwise equal, but measured slower on the 1M P = 3
    // grid (step end 201 us fused against 87 + 61 us as two launches: the
    // quality gathers' registers throttle the whole step-end kernel)
    {
        const char* fq = getenv("SWMM5_FUSE_QUAL");
        d->fuseQual = p.P > 0 && fq && atoi(fq) != 0;
    }
    d->gridEnd = resident((const void*)stepEndKernel(d->fastLinks, d->allShapes, d->fuseQual),
                          std::max(nN, nL));
    p.nBlocksEnd = d->gridEnd;
    {
        std::vector<int> z(d->gridN, 0);
        int* bl;
        UPI(bl, z, d->gridN);
        p.blockLive = bl;
        p.blockLiveN = d->gridN;
    }
    p.multi = part.active() ? 1 : 0;
    // ---- run statistics (stats_open, stats.c:150-240; massbal_open NodeInflow) ----
    {
        StatsDev& S = p.st;
        auto zN = [&](double v) { return std::vector<double>(nN, v); };
        auto zL = [&](double v) { return std::vector<double>(nL, v); };
        std::vector<double> z0 = zN(0.0), l0 = zL(0.0), dStart = zN(prj.opt.startDateTime);
        for (double** a : {&S.avgDepth, &S.maxDepth, &S.volFlooded, &S.timeFlooded, &S.timeSurch,
                           &S.timeCourant, &S.totLat, &S.maxLat, &S.maxInflow, &S.maxOverflow,
                           &S.maxPonded, &S.oAvgFlow, &S.oMaxFlow})
            UPD(*a, z0, nN);
        for (double** a : {&S.maxDepthDate, &S.maxInflowDate, &S.maxOverflowDate}) UPD(*a, dStart, nN);
        std::vector<int> iz(std::max(nN, nL), 0);
        UPI(S.nonConv, iz, nN);
        UPI(S.oPeriods, iz, nN);
        UPI(S.lTurns, iz, nL);
        UPI(S.lTurnSign, iz, nL);
        for (double** a : {&S.lMaxFlow, &S.lMaxFlowDate, &S.lMaxVeloc, &S.lMaxDepth, &S.lTimeNormal, &S.lTimeInlet,
                           &S.lTimeSurch, &S.lTimeFullUp, &S.lTimeFullDn, &S.lTimeFullFlow,
                           &S.lTimeCapLim, &S.lTimeCourant})
            UPD(*a, l0, nL);
        std::vector<double> cls((size_t)7 * nL, 0.0);
        UPD(S.lTimeClass, cls, cls.size());
        for (double** a : {&S.sAvgVol, &S.sMaxVol, &S.sMaxFlow, &S.sEvap, &S.sExfil}) UPD(*a, z0, nN);
        UPD(S.sMaxVolDate, dStart, nN);
        std::vector<double> ol((size_t)std::max(P, 1) * nN, 0.0);
        UPD(S.oLoad, ol, ol.size());
        UPD(tmp, gl(net.qFull), nL); S.qFull = tmp;
        // per-node volume totals start from the initial volume; the pending
        // half-step rates are the initial state's (massbal.c:239, 619-633)
        std::vector<double> vin(nN), pin(nN), pout((size_t)2 * nN);
        for (int i = 0; i < nN; i++) {
            const int g = LN[i];
            vin[i] = st.newVolume[g];
            pin[i] = st.inflow[g];
            bool passthru = net.nodeType[g] == OUTFALL || net.degree[g] == 0;
            pout[i] = passthru ? st.inflow[g] : st.outflow[g];
            pout[nN + i] = (!passthru && st.newVolume[g] <= net.fullVolume[g]) ? st.overflow[g] : 0.0;
        }
        UPD(S.mbIn, vin, nN);
        UPD(S.mbOut, z0, nN);
        UPD(S.mbPendIn, pin, nN);
        UPD(S.mbPendOut, pout, pout.size());
    }
    // ---- multi-GPU exchange ----------------------------------------------------
    p.nSend = (int)part.sendLink.size();
    p.nGhost = (int)part.lghost.size();
    {
        // evaporation / seepage values travel too when any link of the whole
        // network has them (the same count on every rank: what one rank sends
        // another receives)
        bool seep = false;
        for (int g = 0; g < gL && !seep; g++)
            seep = net.seepRate[g] > 0.0 || (prj.evapCanBePositive() && isOpen(net.xsect[g].type));
        p.xF = seep ? 6 : 4;
        const int w = std::max(p.xF, P);
        int* ip;
        UPI(ip, part.sendLink, part.sendLink.size()); p.sendLink = ip;
        std::vector<double> zs((size_t)w * std::max(p.nSend, 1), 0.0), zg((size_t)w * std::max(p.nGhost, 1), 0.0);
        UPD(p.xsend, zs, zs.size());
        UPD(p.xrecv, zg, zg.size());
        d->gridX = std::max(1, std::min((std::max(p.nSend, p.nGhost) + kBlock - 1) / kBlock, maxBlocks));
        p.ipc = 0;
        p.xRank = part.rank;
        p.xRanks = part.nranks;
        p.stallStep = -1;
        p.xwake = 0;
        p.xwlist = nullptr;
        p.xwcount = nullptr;
        if (part.active()) {                        // shared nodes freeze unless SWMM5_SHARED_FREEZE=0
            const char* sf = getenv("SWMM5_SHARED_FREEZE");
            p.xwake = (sf && atoi(sf) == 0) ? 0 : 1;
            p.xwlist = devAlloc<int>(d, (size_t)std::max(nN, 1), &e);
            if (e == hipSuccess) p.xwcount = devAlloc<int>(d, (size_t)std::max(p.maxTrials, 1), &e);
            if (e == hipSuccess) e = hipMemset(p.xwcount, 0, (size_t)std::max(p.maxTrials, 1) * sizeof(int));
            if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
        }
        HIPCHECK(hipHostMalloc((void**)&d->xerrHost, 4 * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHECK(hipHostMalloc((void**)&d->hostAbortH, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
        memset(d->xerrHost, 0, 4 * sizeof(int));
        *d->hostAbortH = 0;
        {
            void* dp = nullptr;
            HIPCHECK(hipHostGetDevicePointer(&dp, d->xerrHost, 0));
            p.xerr = (int*)dp;
            HIPCHECK(hipHostGetDevicePointer(&dp, d->hostAbortH, 0));
            p.hostAbort = (const int*)dp;
        }
        if (const char* ts = getenv("SWMM5_XCHG_TIMEOUT"))
            if (atof(ts) > 0.0) d->xTimeoutSec = atof(ts);
        if (const char* xf = getenv("SWMM5_XCHG_FUSED")) d->xchgFusedEnv = atoi(xf) != 0 ? 1 : 0;
        p.xTimeout = (long long)(d->xTimeoutSec * d->wallKHz * 1000.0);
        if (const char* st = getenv("SWMM5_XCHG_STALL")) {     // test hook "rank:step"
            int r = -1;
            long long s = -1;
            if (sscanf(st, "%d:%lld", &r, &s) == 2 && r == part.rank) p.stallStep = s;
        }
        d->transportName = "single";
        if (part.active()) {
            auto initRccl = [&]() -> bool {
                // single-node bootstrap over the loopback interface unless the
                // caller chose one (an unset interface lets RCCL probe the
                // host's interfaces at communicator creation)
                setenv("NCCL_SOCKET_IFNAME", "lo", 0);
                if (part.ncclId.size() != sizeof(ncclUniqueId)) { fail("RCCL unique id missing"); return false; }
                ncclUniqueId id;
                memcpy(&id, part.ncclId.data(), sizeof id);
                ncclResult_t r = ncclCommInitRank(&d->comm, part.nranks, id, part.rank);
                if (r != ncclSuccess) { fail(std::string("ncclCommInitRank: ") + ncclGetErrorString(r)); return false; }
                return true;
            };
            if (part.transport == XCHG_RCCL) {
                if (!initRccl()) return err_;
                d->transportName = "rccl";
            } else if (part.transport == XCHG_IPC) {
                if (!part.xchg && !initRccl()) return err_;      // bootstrap over RCCL
                const int r = setupIpc(d);
                if (r == 500) { fail(d->xerrMsg); return err_; }
                if (r == 0) {
                    d->transportName = "ipc";
                } else {                                          // not usable here: fall back
                    memset(d->xerrHost, 0, 4 * sizeof(int));
                    *d->hostAbortH = 0;
                    if (part.ncclId.size() == sizeof(ncclUniqueId)) {
                        if (!d->comm && !initRccl()) return err_;
                        d->part.transport = XCHG_RCCL;
                        d->transportName = "rccl (IPC transport unavailable: fell back)";
                    } else if (part.xchg) {
                        d->part.transport = XCHG_HOST;
                        d->transportName = "host (IPC transport unavailable: fell back)";
                    } else {
                        fail("IPC transport unavailable and no fallback transport");
                        return err_;
                    }
                }
            }
            if (d->part.transport == XCHG_HOST) {
                if (!part.xchg) { fail("host exchange callback missing"); return err_; }
                size_t nx = (size_t)w * std::max(p.nSend, p.nGhost) + 8;
                HIPCHECK(hipHostMalloc((void**)&d->hostX, nx * sizeof(double), hipHostMallocDefault));
                if (d->transportName == "single") d->transportName = "host";
            }
        }
    }
    p.partials = devAlloc<double>(d, (size_t)d->gridEnd * kNumPartials, &e);
    if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
    p.ctl = devAlloc<StepCtl>(d, 1, &e);
    if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
    {   // per-iteration flags and counters, sized from MAX_TRIALS (any value the reference accepts)
        const size_t M = (size_t)std::max(p.maxTrials, 1);
        std::vector<int> zi(M, 0);
        UPI(p.unconv, zi, M);
        UPI(p.ucount, zi, M);
        UPI(p.vcount, zi, M);
        UPI(p.wcount, zi, M);
        p.work = devAlloc<unsigned long long>(d, 4 * M, &e);
        if (e == hipSuccess) e = hipMemset(p.work, 0, 4 * M * sizeof(unsigned long long));
        p.probe = nullptr;                         // set in timing mode under SWMM5_PROBE
        p.probeBlocks = 0;
        if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
    }
    d->ctl = p.ctl;
    HIPCHECK(hipHostMalloc((void**)&d->hostCtl, sizeof(StepCtl), hipHostMallocDefault));
    memset(d->hostCtl, 0, sizeof(StepCtl));
    StepCtl* hc = d->hostCtl;
    hc->routeStep = prj.opt.routeStep;
    hc->routingDuration = prj.opt.totalDuration;
    hc->newRoutingTime = 0.0;
    // first step: dynwave_getRoutingStep returns MinRouteStep while VariableStep == 0
    double dt0 = p.varStep ? floor(1000.0 * prj.opt.minRouteStep) / 1000.0 : prj.opt.routeStep;
    if (!p.varStep) { /* fixed step */ }
    if (1000.0 * dt0 > hc->routingDuration) {
        dt0 = hc->routingDuration / 1000.0;
        dt0 = (dt0 >= 1. / 1000.0) ? dt0 : 1. / 1000.0;
    }
    hc->dt = dt0;
    hc->latTot[0] = d->latTot0[0];
    hc->latTot[1] = d->latTot0[1];
    hc->latTot[2] = d->latTot0[2];
    hc->statsStart = prj.opt.reportStart;
    hc->evapRate = prj.opt.evapRate;
    hc->hydconFactor = prj.opt.hydconFactor;
    hc->recoveryFactor = prj.opt.recoveryFactor;
    d->climateDev[0] = prj.opt.evapRate;
    d->climateDev[1] = prj.opt.hydconFactor;
    d->climateDev[2] = prj.opt.recoveryFactor;
    {
        int h, m, sec;
        decodeTime(prj.opt.startDateTime, &h, &m, &sec);
        hc->dateBase = floor(prj.opt.startDateTime);
        hc->dateSecs0 = 3600.0 * h + 60.0 * m + sec;       // datetime_addSeconds' operand order
    }
    // stats_open's time-step intervals (stats.c:288-312)
    hc->tsMax = 0.0;
    hc->tsMin = prj.opt.routeStep;
    {
        double lmax = log10(prj.opt.routeStep), lmin = log10(prj.opt.minRouteStep);
        double delta = (lmax - lmin) / (double)(kTimeLevels - 1);
        hc->tsIntervals[0] = prj.opt.routeStep;
        for (int j = 1; j < kTimeLevels; j++) hc->tsIntervals[j] = pow(10., lmax - j * delta);
        hc->tsIntervals[kTimeLevels - 1] = prj.opt.minRouteStep;
    }
    HIPCHECK(hipMemcpy(d->ctl, d->hostCtl, sizeof(StepCtl), hipMemcpyHostToDevice));
    d->slotDoubles = (size_t)nN * (1 + P) + 8;
    d->pinnedSize = d->slotDoubles * Impl::kRing;
    HIPCHECK(hipHostMalloc((void**)&d->hostPinned, d->pinnedSize * sizeof(double), hipHostMallocDefault));
    for (auto& ev : d->ringEv) { HIPCHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming)); HIPCHECK(hipEventRecord(ev, d->stream)); }
    for (auto& ev : d->clockEv) HIPCHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIPCHECK(hipHostMalloc((void**)&d->hostDt, (3 * Impl::kRing + 1) * sizeof(double),
                           hipHostMallocMapped | hipHostMallocCoherent));
    {
        void* dp = nullptr;
        HIPCHECK(hipHostGetDevicePointer(&dp, d->hostDt, 0));
        p.hostDt = (double*)dp;
        for (int r = 0; r < Impl::kRing; r++) {
            d->hostDt[r] = d->hostCtl->dt;
            d->hostDt[Impl::kRing + r] = 0.0;
            d->hostDt[2 * Impl::kRing + 1 + r] = 0.0;
        }
        d->hostDt[2 * Impl::kRing] = 0.0;          // k_tail barrier timeout flag
    }

    // algorithmic bytes per launch (DESIGN.md byte model; per kernel class)
    {
        double L = nL, N = nN, E = d->nE;
        // link momentum, per streaming conduit:
        //   static   nodes 8 + flags 4 + inv1/inv2 16 + geometry 7x8
        //            + length/modLength/roughFactor/beta 32           = 116
        //   gathers  newDepth at both end nodes                       =  16
        //   writes   a1 q1 newDepth newVolume newFlow dqdh froude
        //            sa1 sa2 evap seep 11x8 + lstate 4                =  92
        //   iteration 0 (k_link<true>): reads newFlow newDepth newVolume a1
        //            setting q1 6x8 + lstate 4, writes oldFlow oldDepth
        //            oldVolume a2 4x8                                 =  84
        //   iterations >= 1: reads oldFlow setting q1 a2 4x8 + lstate 4 = 36
        //   a bypassed conduit costs flags 4 + nodes 8 + 2 conv flags 8 = 20,
        //   a cold conduit skipped by the streaming kernel costs its flags 4
        //   (kFast: the geometry comes from the LDS section table: static 60;
        //   evap and seep are written only by conduits with losses, LF_SEEP)
        d->nHot = L - p.nCold;
        d->nColdD = p.nCold;
        double nSeepHot = 0;
        for (int j = 0; j < nL; j++)
            if (!(lflags[j] & LF_COLD) && (lflags[j] & LF_SEEP)) nSeepHot += 1;
        const double stat = d->fastLinks ? 60 : 116;
        d->kbytes[0] = d->nHot * (stat + 16 + 76 + 84) + nSeepHot * 16 + d->nColdD * 4;
        d->kbytes[4] = stat + 16 + 76 + 36 + (d->nHot > 0 ? 16.0 * nSeepHot / d->nHot : 0.0);
        // node update (k_node), per node, iteration 0: reads flags 4, yLast 8,
        //   rowptr 4 (+ the neighbour's), fullDepth yCrown surDepth fullVolume
        //   32 and the step-begin rotation's inflow outflow newVolume newLat
        //   latIn 40 = 88; writes the rotation's oldDepth oldVolume
        //   oldFlowInflow oldNetInflow oldLat newLat 48, the sums inflow
        //   outflow surfArea sumdqdh 32, oldSurfArea newVolume overflow
        //   newDepth 32 and conv 4 = 116; per CSR entry: index 4 + the link's
        //   newFlow 8, flags 4, surfArea at that end 8, dqdh 8 = 32
        //   iteration 1: no rotation; reads yOld lat oldNetInflow instead
        //   (72), writes the sums, oldSurfArea newVolume overflow newDepth
        //   conv, the cached unrelaxed depth yRaw and the dirty byte (77)
        //   iterations >= 2: every node's flags, frozen and dirty bytes are
        //   scanned (6); a relaxation-only update reads newDepth yCrown yRaw
        //   yMaxNP and writes newDepth conv (44); a full update reads yLast
        //   yOld lat oldNetInflow fullDepth yCrown surDepth fullVolume (64),
        //   writes oldSurfArea newVolume overflow newDepth conv dirty yRaw
        //   (45) and reads or writes the four sums (32); a gathering node
        //   adds rowptr 8 and its CSR entries (32 each).  The counts of each
        //   kind come from the timing-mode counters (StepCtl nodeLive /
        //   nodeFast / nodeWork), so frozen nodes are not charged bytes they
        //   never fetch.
        d->kbytes[1] = N * (88 + 116) + E * 32;
        d->nodeIter1 = N * (72 + 77) + E * 32;
        d->nodeScan = 6;
        d->nodeFastB = 44;
        d->nodeUpdB = 64 + 45 + 32;
        d->nodeGather = 8 + (N > 0 ? (double)E / N * 32.0 : 0.0);
        d->kbytes[5] = d->nodeIter1;
        d->kbytes[6] = N * (6 + 141) + E * 32;    // every node updated and gathering (no timing data)
        // step end: per conduit flags, state word (r+w), a1, aFull, newFlow,
        //   froude, newVolume, modLength, length (48 + 4) and the run
        //   statistics: oldFlow, maxFlow, newDepth, maxVeloc, maxDepth, the
        //   flow-class time (r+w), qFull, turn sign (r+w) (96): 148; per node
        //   flags, inflow, outflow, overflow, volumes, depths, crown, invert,
        //   dYdT (84), the volume totals and pending rates (r+w, 80), the node
        //   statistics avgDepth (r+w), maxDepth, newLat, oldLat, totLat (r+w),
        //   maxLat, maxInflow, maxOverflow, conv (96): 260 (conditional
        //   updates of maxima and times not counted)
        d->kbytes[2] = L * 148.0 + N * 260.0;
        // quality (k_qual_node): per node depth inflow oldVolume newVolume
        //   flags qrowptr 40 + loads, old and new concentration 24 P; per CSR
        //   entry index 4 + newFlow 8 + a downstream link's concentration 8 P
        //   (half the entries); per link its update: flags q1 seep evap
        //   volumes depth 52, old and new concentration 16 P
        d->kbytes[3] = P ? (N * (40 + 24.0 * P) + E * (12 + 4.0 * P) + L * (52 + 16.0 * P)) : 0.0;
    }

    {   // the outfall conduits' enumeration critical flows (static)
        double* q = devAlloc<double>(d, 26 * (size_t)std::max(p.nOutLinks, 1), &e);
        if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
        if (p.nOutLinks > 0) {
            hipLaunchKernelGGL(k_outfall_qcs, dim3((26 * p.nOutLinks + kBlock - 1) / kBlock), dim3(kBlock), 0,
                               d->stream, p, q);
            HIPCHECK(hipGetLastError());
            WAITCHECK(waitDone(d_, nullptr));
        }
        p.ofQcs = q;
    }

    // ---- capture the step graph ----------------------------------------------
    // (the host-callback test transport synchronises inside the step: eager)
    d->useGraph = !(part.active() && part.transport == XCHG_HOST);
    if (!d->useGraph) {
        // eager launches: the per-step choice between the unrolled and the
        // list graph's launch sequences (the others are single-GPU)
        const char* sm = getenv("SWMM5_SPARSE");
        d->sparseMode = sm ? atoi(sm) : 2;
        if (const char* lx = getenv("SWMM5_LIST_MAX")) d->listMax = atof(lx);
        d->listOk = d->sparseMode != 0 && p.maxTrials > 2;
        ok_ = true;
        return 0;
    }
    {
        // off by default: on the surcharged 1M grid (round 4) the walk with the
        // prologue took longer than the node launch saved (SWMM5_DEFER_OUTFALL=1
        // turns it on)
        const char* dp = getenv("SWMM5_DEFER_OUTFALL");
        const char* es = getenv("SWMM5_STEPEND_SKIP");
        p.endSkip = es ? atoi(es) : 0;
        p.deferPro = (outfallsDeferrable && dp && atoi(dp) != 0 && !part.active() && !d->comm && p.nNC == 0 &&
                      p.maxTrials > 2) ? 1 : 0;
    }
    hipGraph_t g;
    HIPCHECK(hipStreamBeginCapture(d->stream, hipStreamCaptureModeThreadLocal));
    if (launchStep(d)) {                           // a collective refused at capture
        (void)hipStreamEndCapture(d->stream, &g);
        fail(d->xerrMsg);
        return err_;
    }
    HIPCHECK(hipStreamEndCapture(d->stream, &g));
    HIPCHECK(hipGraphInstantiate(&d->graph, g, nullptr, nullptr, 0));
    (void)hipGraphDestroy(g);
    // the k_tail variant: single GPU, no pumps/regulators (k_nc runs between
    // the node update and the next link update), at least three iterations;
    // one workgroup per CU (all resident: checked against the occupancy)
    {
        const char* tm = getenv("SWMM5_TAIL");
        d->tailMode = tm ? atoi(tm) : 2;
        int occ = 0, cus = 0;
        bool ok = d->tailMode != 0 && !part.active() && !d->comm && p.nNC == 0 && p.maxTrials > 2;
        if (ok && (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
                   hipOccupancyMaxActiveBlocksPerMultiprocessor(
                       &occ, (const void*)tailKernel(d->fastLinks, d->general), kBlock, 0) != hipSuccess))
            ok = false;
        (void)hipGetLastError();
        const char* tw = getenv("SWMM5_TAIL_PER_CU");
        int perCU = std::max(1, std::min(tw ? atoi(tw) : 1, occ - 1 > 0 ? occ - 1 : 1));
        d->tailGrid = (ok && occ >= 1 && cus > 0) ? perCU * cus : 0;
        // a smaller resident grid (SWMM5_TAIL_GRID workgroups): fewer barrier
        // arrivals when the iterations' lists are short
        if (const char* tg = getenv("SWMM5_TAIL_GRID"))
            if (d->tailGrid > 0 && atoi(tg) > 0) d->tailGrid = std::min(d->tailGrid, atoi(tg));
    }
    if (d->tailGrid > 0) {
        HIPCHECK(hipStreamBeginCapture(d->stream, hipStreamCaptureModeThreadLocal));
        if (launchStep(d, GM_TAIL)) {
            (void)hipStreamEndCapture(d->stream, &g);
            fail(d->xerrMsg);
            return err_;
        }
        HIPCHECK(hipStreamEndCapture(d->stream, &g));
        HIPCHECK(hipGraphInstantiate(&d->graphTail, g, nullptr, nullptr, 0));
        (void)hipGraphDestroy(g);
    }
    // the k_sparse variant: the same conditions as k_tail (single GPU, no
    // pumps / regulators, at least three iterations), one workgroup
    {
        const char* sm = getenv("SWMM5_SPARSE");
        d->sparseMode = sm ? atoi(sm) : 2;
        if (const char* sx = getenv("SWMM5_SPARSE_MAX")) d->sparseMax = atof(sx);
        if (const char* lx = getenv("SWMM5_LIST_MAX")) d->listMax = atof(lx);
        d->sparseOk = d->sparseMode != 0 && !part.active() && !d->comm && p.nNC == 0 && p.maxTrials > 2;
        d->listOk = d->sparseMode != 0 && p.maxTrials > 2;
    }
    if (d->sparseOk) {
        HIPCHECK(hipStreamBeginCapture(d->stream, hipStreamCaptureModeThreadLocal));
        if (launchStep(d, GM_SPARSE)) {
            (void)hipStreamEndCapture(d->stream, &g);
            fail(d->xerrMsg);
            return err_;
        }
        HIPCHECK(hipStreamEndCapture(d->stream, &g));
        HIPCHECK(hipGraphInstantiate(&d->graphSparse, g, nullptr, nullptr, 0));
        (void)hipGraphDestroy(g);
    }
    if (d->listOk) {
        HIPCHECK(hipStreamBeginCapture(d->stream, hipStreamCaptureModeThreadLocal));
        if (launchStep(d, GM_LIST)) {
            (void)hipStreamEndCapture(d->stream, &g);
            fail(d->xerrMsg);
            return err_;
        }
        HIPCHECK(hipStreamEndCapture(d->stream, &g));
        HIPCHECK(hipGraphInstantiate(&d->graphList, g, nullptr, nullptr, 0));
        (void)hipGraphDestroy(g);
    }
    WAITCHECK(waitDone(d_, nullptr));
    ok_ = true;
    return 0;
#undef UPD
#undef UPI
}

// Accumulate the per-kernel-class times of all pending timed steps.
// SWMM5_PROBE (timing mode): read the step's per-workgroup phase stamps back
// (synchronously: a measurement run), fold them into per-iteration phase
// times relative to the link kernel's first workgroup start, and clear them
static void probeCollect(Router::Impl* d)
{
    const Params& p = d->p;
    const int M = std::max(p.maxTrials, 1), B = p.probeBlocks;
    std::vector<unsigned long long> h((size_t)M * kProbeSlots * B);
    if (hipMemcpyAsync(h.data(), p.probe, h.size() * sizeof(h[0]), hipMemcpyDeviceToHost, d->stream) != hipSuccess ||
        hipStreamSynchronize(d->stream) != hipSuccess)
        return;
    (void)hipMemsetAsync(p.probe, 0, h.size() * sizeof(h[0]), d->stream);
    const int C = kProbeSlots + 7;
    if (d->probeSum.size() < (size_t)C * M) d->probeSum.assign((size_t)C * M, 0.0);
    const double us = 1000.0 / d->wallKHz;
    for (int k = 0; k < M; k++) {
        auto slot = [&](int sl, bool mx, bool b0) {
            const unsigned long long* q = h.data() + ((size_t)kProbeSlots * k + sl) * B;
            if (b0) return (double)q[0];
            unsigned long long v = mx ? 0ull : ~0ull;
            for (int b = 0; b < B; b++)
                if (q[b]) v = mx ? std::max(v, q[b]) : std::min(v, q[b]);
            return (v == 0ull || v == ~0ull) ? 0.0 : (double)v;
        };
        const double l0 = slot(PR_L_IN, false, false), n0 = slot(PR_N_IN, false, false);
        if (l0 == 0.0 || n0 == 0.0) continue;          // iteration k did not run
        double* o = d->probeSum.data() + (size_t)C * k;
        o[PR_L_IN] += (slot(PR_L_IN, true, false) - l0) * us;         // last link workgroup's start
        o[PR_L_OUT] += (slot(PR_L_OUT, true, false) - l0) * us;
        const double w = slot(PR_L_WORK, true, false);
        if (w > 0.0) o[PR_L_WORK] += (w - l0) * us;
        o[PR_N_IN] += (n0 - l0) * us;
        o[PR_N_LAST_IN] += (slot(PR_N_LAST_IN, true, false) - l0) * us;
        const double pr = slot(PR_N_PRO, true, true);
        if (pr > 0.0) o[PR_N_PRO] += (pr - l0) * us;
        o[PR_N_OUT] += (slot(PR_N_OUT, true, false) - l0) * us;
        o[PR_N_B0] += (slot(PR_N_B0, true, true) - l0) * us;
        for (int sl : {PR_P_STAGED, PR_P_YN, PR_P_YC}) {
            const double v = slot(sl, true, true);
            if (v > 0.0) o[sl] += (v - l0) * us;
        }
        {   // link workgroups with list work: median phase times after their own start
            const unsigned long long* a = h.data() + ((size_t)kProbeSlots * k + PR_L_IN) * B;
            std::vector<double> ph[3];
            const int sl[3] = {PR_L_SCAN, PR_L_STAGED, PR_L_WORK};
            for (int x = 0; x < 3; x++) {
                const unsigned long long* z = h.data() + ((size_t)kProbeSlots * k + sl[x]) * B;
                for (int b = 0; b < B; b++)
                    if (a[b] && z[b]) ph[x].push_back((double)(z[b] - a[b]) * us);
                if (!ph[x].empty()) {
                    std::sort(ph[x].begin(), ph[x].end());
                    o[kProbeSlots + 4 + x] += ph[x][ph[x].size() / 2];
                }
            }
        }
        {   // per-workgroup node kernel durations: median, maximum, slowest workgroup
            const unsigned long long* a = h.data() + ((size_t)kProbeSlots * k + PR_N_IN) * B;
            const unsigned long long* z = h.data() + ((size_t)kProbeSlots * k + PR_N_OUT) * B;
            std::vector<std::pair<double, int>> dur;
            for (int b = 0; b < B; b++)
                if (a[b] && z[b]) dur.push_back({(double)(z[b] - a[b]) * us, b});
            if (!dur.empty()) {
                std::sort(dur.begin(), dur.end());
                o[kProbeSlots + 1] += dur[dur.size() / 2].first;
                o[kProbeSlots + 2] += dur.back().first;
                o[kProbeSlots + 3] = dur.back().second;
            }
        }
        o[kProbeSlots] += 1;
    }
}

static void flushTiming(Router::Impl* d)
{
    if (!d->tUsed) return;
    (void)waitDone(d, nullptr);
    const Params& p = d->p;
    for (int s = 0; s < d->tUsed; s++) {
        Router::Impl::TimingSlot& t = d->tslots[s];
        int ran = (int)(t.pinned[0] & 0xFFFFFFFFull);
        const unsigned long long* work = t.pinned + 1;       // linkWork, nodeWork, nodeLive, nodeFast
        if ((int)d->iterStats.size() < Router::Impl::kIterCols * p.maxTrials)
            d->iterStats.assign((size_t)Router::Impl::kIterCols * p.maxTrials, 0.0);
        const bool sparse = t.mode == GM_SPARSE;
        if (sparse) {                      // iterations k >= 2: one k_sparse + k_unfreeze pair
            float ms = 0;
            (void)hipEventElapsedTime(&ms, t.ev[4 * p.maxTrials + 4], t.ev[4 * p.maxTrials + 5]);
            d->kms[7] += ms; d->kcnt[7]++;
        }
        for (int k = 0; k < ran; k++) {    // early-exited iterations are not counted
            float ms1 = 0, ms2 = 0;
            if (k >= 1) d->itersTimed1++;
            if (sparse && k >= 2) {        // work counters only (no per-iteration events)
                const int M = p.maxTrials;
                double* it = d->iterStats.data() + (size_t)Router::Impl::kIterCols * k;
                it[0] += 1;
                it[1] += (double)work[k];
                it[2] += (double)work[M + k];
                it[3] += (double)work[2 * M + k];
                it[4] += (double)work[3 * M + k];
                d->workSum += (double)work[k];
                d->gatherSum += (double)work[M + k]; d->gatherCnt += 1;
                continue;
            }
            (void)hipEventElapsedTime(&ms1, t.ev[4 * k], t.evHot[k]);
            (void)hipEventElapsedTime(&ms2, t.ev[4 * k + 1], t.ev[4 * k + 2]);
            {
                const int M = p.maxTrials;
                double* it = d->iterStats.data() + (size_t)Router::Impl::kIterCols * k;
                it[0] += 1;
                it[1] += (k >= 2) ? (double)work[k] : d->nHot;
                it[2] += (k >= 2) ? (double)work[M + k] : (double)p.nN;
                it[3] += (k >= 2) ? (double)work[2 * M + k] : (double)p.nN;
                it[4] += (k >= 2) ? (double)work[3 * M + k] : 0.0;
                it[5] += ms1;
                it[6] += ms2;
            }
            int c = (k == 0) ? 0 : 4;
            d->kms[c] += ms1; d->kcnt[c]++;
            if (k == 0) d->kbytesSum[0] += d->kbytes[0];
            else {
                double w = (k >= 2) ? (double)work[k] : d->nHot;   // no bypass before iteration 2
                d->workSum += w;
                d->kbytesSum[4] += w * d->kbytes[4] + (d->nHot - w) * 20.0 + d->nColdD * 4.0;
            }
            const int cn = (k == 0) ? 1 : (k == 1 ? 5 : 6);
            d->kms[cn] += ms2; d->kcnt[cn]++;
            if (!t.evX.empty()) {                  // several ranks: the two exchanges of iteration k
                float mx = 0, mf = 0;
                (void)hipEventElapsedTime(&mx, t.evX[4 * k], t.evX[4 * k + 1]);
                (void)hipEventElapsedTime(&mf, t.evX[4 * k + 2], t.evX[4 * k + 3]);
                d->kms[8] += mx; d->kcnt[8]++;
                d->kms[9] += mf; d->kcnt[9]++;
            }
            if (k == 0) d->kbytesSum[1] += d->kbytes[1];
            else if (k == 1) d->kbytesSum[5] += d->nodeIter1;
            else {
                const int M = p.maxTrials;
                double g = (double)work[M + k];
                double live = (double)work[2 * M + k], fast = (double)work[3 * M + k];
                d->kbytesSum[6] += d->nodeScan * (double)p.nN + fast * d->nodeFastB +
                                   (live - fast) * d->nodeUpdB + g * d->nodeGather;
                d->gatherSum += g; d->gatherCnt += 1;
            }
        }
        int base = 4 * p.maxTrials;
        float ms3 = 0, msq = 0;
        (void)hipEventElapsedTime(&ms3, t.ev[base + 2], t.ev[base + 3]);
        d->kms[2] += ms3; d->kcnt[2]++;
        d->kbytesSum[2] += d->kbytes[2];
        if (p.P && !d->fuseQual) {
            (void)hipEventElapsedTime(&msq, t.ev[base], t.ev[base + 1]);
            d->kms[3] += msq; d->kcnt[3]++; d->kbytesSum[3] += d->kbytes[3];
        }
    }
    d->tUsed = 0;
}

// Unrolled or k_tail graph for the next step.  Auto: k_tail while the recent
// steps ran few Picard iterations (the unrolled graph's dispatches of the
// iterations that do not run dominate), the unrolled graph otherwise.  The
// iteration counts come from the host-mapped ring k_finalize writes (steps
// already complete; no synchronisation).  Both graphs run the same code on
// the same data: the choice changes no result.
// Sparse graph: while the live lists after iteration 1 (k_finalize writes
// their length into the same ring) average at most sparseMax nodes, when the
// steps run more iterations than k_tail suits.
static int chooseGraph(Router::Impl* d)
{
    constexpr int R = Router::Impl::kRing;
    long long done = d->launched - 2;              // steps surely past their k_finalize?
    while (d->itersSeen < done) {
        long long n = d->itersSeen + 1;
        if (n < 0) { d->itersSeen = n; continue; }
        if (hipEventQuery(d->clockEv[n % R]) != hipSuccess) break;
        const double it = d->hostDt[R + n % R], lv = d->hostDt[2 * R + 1 + n % R];
        d->itersAvg = (d->itersSeen < 0) ? it : 0.9 * d->itersAvg + 0.1 * it;
        d->liveAvg = (d->itersSeen < 0) ? lv : 0.9 * d->liveAvg + 0.1 * lv;
        d->itersSeen = n;
    }
    const bool fresh = d->itersSeen < 0;
    // several ranks: the same graph on every rank at every step, whatever each
    // rank's own live lists (the choice must not depend on the timing of a
    // non-blocking event query); the list graph unless it is turned off
    if (d->part.active()) return d->listOk ? GM_LIST : GM_UNROLLED;
    if (d->sparseOk && d->sparseMode == 1) return GM_SPARSE;
    if (d->listOk && d->sparseMode == 3) return GM_LIST;
    if (d->tailGrid > 0 && (d->tailMode == 1 || fresh || d->itersAvg <= kTailIters)) return GM_TAIL;
    if (d->sparseOk && !fresh && d->liveAvg <= d->sparseMax) return GM_SPARSE;
    if (d->listOk && !fresh && d->liveAvg <= d->listMax) return GM_LIST;
    return GM_UNROLLED;
}

// A k_tail launch whose grid barrier timed out left its step incomplete; the
// flag arrives through the host-mapped ring (k_finalize writes it with a
// system-scope fence).  It is read here without waiting for the step, so
// the failure is reported by the first swmm_step that starts after the
// flag became visible (at the latest, the one after launchedDt or a
// synchronising call observed that step's completion), and k_tail is not
// used again.
static bool tailFailed(Router::Impl* d)
{
    if (d->hostDt[2 * Router::Impl::kRing] == 0.0) return false;
    d->tailGrid = 0;
    return true;
}

int Router::step(const double* latFlow, const double* qualLoad, const double tot[3])
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    Params& p = d->p;
    if (tailFailed(d)) {
        fail("k_tail grid barrier timed out (workgroups not co-resident); the step it ran is incomplete");
        return err_;
    }
    {   // XCHG_IPC: a wait of an earlier step gave up (the record is host-mapped)
        std::string m;
        if (ipcFailed(d, &m)) { fail(m); return err_; }
    }
    if (latFlow) {
        // pinned ring slot: wait until the DMA that last read this slot is done
        int s = d->ringNext;
        d->ringNext = (d->ringNext + 1) % Impl::kRing;
        WAITCHECK(waitDone(d_, d->ringEv[s]));
        double* slot = d->hostPinned + (size_t)s * d->slotDoubles;
        size_t nN = p.nN, nq = (size_t)p.P * nN;
        const Partition& part = d->part;
        if (part.active()) {                       // this rank's held nodes (every replica adds them)
            for (size_t i = 0; i < nN; i++) slot[i] = latFlow[part.lnode[i]];
        } else {
            memcpy(slot, latFlow, nN * sizeof(double));
        }
        if (nq) {
            if (!qualLoad) memset(slot + nN, 0, nq * sizeof(double));
            else if (!part.active()) memcpy(slot + nN, qualLoad, nq * sizeof(double));
            else {                                 // [p][global node] -> [p][held node]
                const size_t gN = part.nodeOwner.size();
                for (size_t q = 0; q < (size_t)p.P; q++)
                    for (size_t i = 0; i < nN; i++) slot[nN + q * nN + i] = qualLoad[q * gN + part.lnode[i]];
            }
        }
        bool countTotals = part.rank == 0;         // system totals counted once
        slot[nN + nq + 0] = countTotals ? tot[0] : 0.0;
        slot[nN + nq + 1] = countTotals ? tot[1] : 0.0;
        slot[nN + nq + 2] = countTotals ? tot[2] : 0.0;
        HIPCHECK(hipMemcpyAsync(d->latBase, slot, nN * sizeof(double), hipMemcpyHostToDevice, d->stream));
        if (nq)
            HIPCHECK(hipMemcpyAsync(d->qualBase, slot + nN, nq * sizeof(double), hipMemcpyHostToDevice, d->stream));
        HIPCHECK(hipMemcpyAsync(&d->ctl->latTot[0], slot + nN + nq, 3 * sizeof(double),
                                hipMemcpyHostToDevice, d->stream));
        HIPCHECK(hipEventRecord(d->ringEv[s], d->stream));
    }
    if (d->timing) {
        // eager launches with a private event set per step; nothing synchronises
        // until the results are read (flushTiming), so steps run back to back
        if (d->tUsed == (int)d->tslots.size() && d->tslots.size() >= 256) flushTiming(d);
        if (d->tUsed == (int)d->tslots.size()) {
            d->tslots.emplace_back();
            Impl::TimingSlot& t = d->tslots.back();
            const int M = std::max(p.maxTrials, 1);
            t.ev.resize(4 * M + 6);
            t.evHot.resize(M);
            if (d->part.active()) t.evX.resize(4 * (size_t)M);
            for (auto& ev : t.evX) HIPCHECK(hipEventCreate(&ev));
            for (auto& ev : t.ev) HIPCHECK(hipEventCreate(&ev));
            for (auto& ev : t.evHot) HIPCHECK(hipEventCreate(&ev));
            HIPCHECK(hipHostMalloc((void**)&t.pinned, (1 + 4 * (size_t)M) * sizeof(unsigned long long),
                                   hipHostMallocDefault));
        }
        Impl::TimingSlot& t = d->tslots[d->tUsed++];
        d->curEv = t.ev.data();
        d->curHot = t.evHot.data();
        d->curX = t.evX.empty() ? nullptr : t.evX.data();
        // the sparse tail when the graphs would run it (k_tail steps are
        // timed as the unrolled sequence)
        t.mode = d->useGraph ? chooseGraph(d) : GM_UNROLLED;
        if (t.mode == GM_TAIL) t.mode = GM_UNROLLED;
        d->modeSteps[t.mode]++;
        if (launchStep(d, t.mode)) { fail(d->xerrMsg); return err_; }
        HIPCHECK(hipMemcpyAsync(t.pinned, &d->ctl->lastSteps, sizeof(int), hipMemcpyDeviceToHost,
                                d->stream));
        const size_t wb = 4 * (size_t)std::max(p.maxTrials, 1) * sizeof(unsigned long long);
        HIPCHECK(hipMemcpyAsync(t.pinned + 1, p.work, wb, hipMemcpyDeviceToHost, d->stream));
        HIPCHECK(hipMemsetAsync(p.work, 0, wb, d->stream));
        if (p.probe) probeCollect(d);
    } else if (d->useGraph) {
        const int mode = chooseGraph(d);
        d->modeSteps[mode]++;
        HIPCHECK(hipGraphLaunch(mode == GM_SPARSE    ? d->graphSparse
                                : mode == GM_LIST    ? d->graphList
                                : mode == GM_TAIL    ? d->graphTail
                                                     : d->graph,
                                d->stream));
    } else {                                       // eager (host-transport exchange)
        const int mode = chooseGraph(d);
        d->modeSteps[mode]++;
        if (launchStep(d, mode)) {
            fail(d->xerrMsg);
            return err_;
        }
    }
    // completion marker of this step: k_finalize has by then written the next
    // step's dt into the host-mapped ring (Router::launchedDt)
    HIPCHECK(hipEventRecord(d->clockEv[d->launched % Impl::kRing], d->stream));
    d->launched++;
    return 0;
}

int Router::launchedDt(double* dt)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    // the step just launched is L-1; its dt was written by step L-2's
    // k_finalize into slot (L-1) % kRing (slot 0 holds the initial step)
    long long L = d->launched;
    if (L >= 2) WAITCHECK(waitDone(d_, d->clockEv[(L - 2) % Impl::kRing]));
    if (tailFailed(d)) {
        fail("k_tail grid barrier timed out (workgroups not co-resident); the step it ran is incomplete");
        return err_;
    }
    *dt = d->hostDt[(L - 1) % Impl::kRing];
    return 0;
}

int Router::readClock(double* t, double* lastDt, double* nextDt)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    HIPCHECK(hipMemcpyAsync(d->hostCtl, d->ctl, sizeof(StepCtl), hipMemcpyDeviceToHost, d->stream));
    WAITCHECK(waitDone(d_, nullptr));
    if (t) *t = d->hostCtl->newRoutingTime;
    if (nextDt) *nextDt = d->hostCtl->dt;
    if (lastDt) *lastDt = d->lastDtHost;
    return 0;
}

int Router::sync()
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    WAITCHECK(waitDone(d_, nullptr));
    return 0;
}

int Router::download(Project& prj)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    Params& p = d->p;
    State& st = prj.st;
    const Partition& part = d->part;
    const bool multi = part.active();
    size_t nN = p.nN, nL = p.nL;
    std::vector<double> tmp;
    // one GPU: straight into the host mirror; several: this rank's owned
    // nodes and its conduits are scattered to their global positions
    auto dnN = [&](std::vector<double>& v, const double* src) -> hipError_t {
        if (!multi) {
            v.resize(nN);
            return hipMemcpyAsync(v.data(), src, nN * sizeof(double), hipMemcpyDeviceToHost, d->stream);
        }
        tmp.resize(nN);
        hipError_t r = hipMemcpy(tmp.data(), src, nN * sizeof(double), hipMemcpyDeviceToHost);
        for (size_t i = 0; i < nN; i++)
            if (part.owned[i]) v[part.lnode[i]] = tmp[i];
        return r;
    };
    auto dnL = [&](std::vector<double>& v, const double* src) -> hipError_t {
        if (!multi) {
            v.resize(nL);
            return hipMemcpyAsync(v.data(), src, nL * sizeof(double), hipMemcpyDeviceToHost, d->stream);
        }
        tmp.resize(nL);
        hipError_t r = hipMemcpy(tmp.data(), src, nL * sizeof(double), hipMemcpyDeviceToHost);
        for (size_t j = 0; j < nL; j++) v[part.llink[j]] = tmp[j];
        return r;
    };
    HIPCHECK(dnN(st.newDepth, p.nNewDepth));
    HIPCHECK(dnN(st.oldDepth, p.nOldDepth));
    HIPCHECK(dnN(st.newVolume, p.nNewVolume));
    HIPCHECK(dnN(st.oldVolume, p.nOldVolume));
    HIPCHECK(dnN(st.inflow, p.inflow));
    HIPCHECK(dnN(st.outflow, p.outflow));
    HIPCHECK(dnN(st.overflow, p.overflow));
    HIPCHECK(dnN(st.newLatFlow, p.newLat));
    HIPCHECK(dnN(st.oldLatFlow, p.oldLat));
    HIPCHECK(dnN(st.oldNetInflow, p.oldNetInflow));
    HIPCHECK(dnN(st.oldFlowInflow, p.oldFlowInflow));
    HIPCHECK(dnN(st.oldSurfArea, p.oldSurfArea));
    HIPCHECK(dnN(st.dYdT, p.dYdT));
    HIPCHECK(dnN(st.hrt, p.hrt));
    HIPCHECK(dnL(st.lNewFlow, p.lNewFlow));
    HIPCHECK(dnL(st.lOldFlow, p.lOldFlow));
    HIPCHECK(dnL(st.lNewDepth, p.lNewDepth));
    HIPCHECK(dnL(st.lOldDepth, p.lOldDepth));
    HIPCHECK(dnL(st.lNewVolume, p.lNewVolume));
    HIPCHECK(dnL(st.lOldVolume, p.lOldVolume));
    HIPCHECK(dnL(st.a1, p.a1));
    HIPCHECK(dnL(st.a2, p.a2));
    HIPCHECK(dnL(st.q1, p.q1));
    HIPCHECK(dnL(st.dqdh, p.dqdh));
    HIPCHECK(dnL(st.froude, p.froude));
    HIPCHECK(dnL(st.surfArea1, p.sa1));
    HIPCHECK(dnL(st.surfArea2, p.sa2));
    HIPCHECK(dnL(st.evapLossRate, p.evapLoss));
    HIPCHECK(dnL(st.seepLossRate, p.seepLoss));
    HIPCHECK(dnL(st.setting, p.setting));
    size_t P = p.P;
    int qp = 0;                                     // the buffer holding the latest concentrations
    if (P) {
        HIPCHECK(hipMemcpyAsync(&d->hostCtl->qualPar, &d->ctl->qualPar, sizeof(int), hipMemcpyDeviceToHost,
                                d->stream));
        WAITCHECK(waitDone(d_, nullptr));
        qp = d->hostCtl->qualPar;
    }
    if (P && !multi) {
        auto dn = [&](std::vector<double>& v, const double* src, size_t n) {
            v.resize(n);
            return hipMemcpyAsync(v.data(), src, n * sizeof(double), hipMemcpyDeviceToHost, d->stream);
        };
        HIPCHECK(dn(st.nOldQual, p.nQual[qp ^ 1], P * nN));
        HIPCHECK(dn(st.nNewQual, p.nQual[qp], P * nN));
        HIPCHECK(dn(st.lOldQual, p.lQual[qp ^ 1], P * nL));
        HIPCHECK(dn(st.lNewQual, p.lQual[qp], P * nL));
    } else if (P) {                                 // owned nodes / links to their global slots
        const size_t gN = prj.net.nNodes(), gL = prj.net.nLinks(), nLs = p.nLs;
        auto qn = [&](std::vector<double>& v, const double* src) -> hipError_t {
            v.resize(P * gN);
            tmp.resize(P * nN);
            hipError_t r = hipMemcpy(tmp.data(), src, P * nN * sizeof(double), hipMemcpyDeviceToHost);
            for (size_t q = 0; q < P; q++)
                for (size_t i = 0; i < nN; i++)
                    if (part.owned[i]) v[q * gN + part.lnode[i]] = tmp[q * nN + i];
            return r;
        };
        auto ql = [&](std::vector<double>& v, const double* src) -> hipError_t {
            v.resize(P * gL);
            tmp.resize(P * nLs);
            hipError_t r = hipMemcpy(tmp.data(), src, P * nLs * sizeof(double), hipMemcpyDeviceToHost);
            for (size_t q = 0; q < P; q++)
                for (size_t j = 0; j < nL; j++) v[q * gL + part.llink[j]] = tmp[q * nLs + j];
            return r;
        };
        HIPCHECK(qn(st.nOldQual, p.nQual[qp ^ 1]));
        HIPCHECK(qn(st.nNewQual, p.nQual[qp]));
        HIPCHECK(ql(st.lOldQual, p.lQual[qp ^ 1]));
        HIPCHECK(ql(st.lNewQual, p.lQual[qp]));
    }
    std::vector<int> ls(nL), cv(nN);
    HIPCHECK(hipMemcpyAsync(ls.data(), p.lstate, nL * sizeof(int), hipMemcpyDeviceToHost, d->stream));
    HIPCHECK(hipMemcpyAsync(cv.data(), p.conv, nN * sizeof(int), hipMemcpyDeviceToHost, d->stream));
    HIPCHECK(hipMemcpyAsync(d->hostCtl, d->ctl, sizeof(StepCtl), hipMemcpyDeviceToHost, d->stream));
    WAITCHECK(waitDone(d_, nullptr));
    size_t gL = multi ? prj.net.nLinks() : nL, gN = multi ? prj.net.nNodes() : nN;
    st.flowClass.resize(gL); st.fullState.resize(gL); st.normalFlow.resize(gL); st.capacityLimited.resize(gL);
    st.converged.resize(gN);
    for (size_t j = 0; j < nL; j++) {
        size_t g = multi ? part.llink[j] : j;
        st.flowClass[g] = ls[j] & 0xF;
        st.fullState[g] = (ls[j] >> 4) & 0xF;
        st.normalFlow[g] = (ls[j] >> 8) & 1;
        st.capacityLimited[g] = (ls[j] >> 9) & 1;
    }
    for (size_t i = 0; i < nN; i++)
        if (!multi || part.owned[i]) st.converged[multi ? part.lnode[i] : i] = cv[i];
    st.variableStep = d->hostCtl->variableStep;
    return 0;
}

int Router::downloadStats(Project& prj)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    const Params& p = d->p;
    const StatsDev& S = p.st;
    const Partition& part = d->part;
    const bool multi = part.active();
    RunStats& R = prj.stats;
    const size_t nN = p.nN, nL = p.nL, gN = prj.net.nNodes(), gL = prj.net.nLinks();
    std::vector<double> tmp;
    std::vector<int> itmp;
    auto node = [&](std::vector<double>& out, const double* src) -> hipError_t {
        out.assign(gN, 0.0);
        tmp.resize(nN);
        hipError_t e = hipMemcpy(tmp.data(), src, nN * sizeof(double), hipMemcpyDeviceToHost);
        for (size_t i = 0; i < nN; i++)
            if (!multi || part.owned[i]) out[multi ? part.lnode[i] : i] = tmp[i];
        return e;
    };
    auto nodeI = [&](std::vector<double>& out, const int* src) -> hipError_t {
        out.assign(gN, 0.0);
        itmp.resize(nN);
        hipError_t e = hipMemcpy(itmp.data(), src, nN * sizeof(int), hipMemcpyDeviceToHost);
        for (size_t i = 0; i < nN; i++)
            if (!multi || part.owned[i]) out[multi ? part.lnode[i] : i] = itmp[i];
        return e;
    };
    auto link = [&](std::vector<double>& out, const double* src, size_t rows) -> hipError_t {
        out.assign(rows * gL, 0.0);
        tmp.resize(rows * nL);
        hipError_t e = hipMemcpy(tmp.data(), src, rows * nL * sizeof(double), hipMemcpyDeviceToHost);
        for (size_t r = 0; r < rows; r++)
            for (size_t j = 0; j < nL; j++) out[r * gL + (multi ? part.llink[j] : j)] = tmp[r * nL + j];
        return e;
    };
    auto linkI = [&](std::vector<double>& out, const int* src) -> hipError_t {
        out.assign(gL, 0.0);
        itmp.resize(nL);
        hipError_t e = hipMemcpy(itmp.data(), src, nL * sizeof(int), hipMemcpyDeviceToHost);
        for (size_t j = 0; j < nL; j++) out[multi ? part.llink[j] : j] = itmp[j];
        return e;
    };
    WAITCHECK(waitDone(d_, nullptr));
    HIPCHECK(node(R.avgDepth, S.avgDepth));
    HIPCHECK(node(R.maxDepth, S.maxDepth));
    HIPCHECK(node(R.maxDepthDate, S.maxDepthDate));
    HIPCHECK(node(R.volFlooded, S.volFlooded));
    HIPCHECK(node(R.timeFlooded, S.timeFlooded));
    HIPCHECK(node(R.timeSurcharged, S.timeSurch));
    HIPCHECK(node(R.timeCourantCritical, S.timeCourant));
    HIPCHECK(node(R.totLatFlow, S.totLat));
    HIPCHECK(node(R.maxLatFlow, S.maxLat));
    HIPCHECK(node(R.maxInflow, S.maxInflow));
    HIPCHECK(node(R.maxInflowDate, S.maxInflowDate));
    HIPCHECK(node(R.maxOverflow, S.maxOverflow));
    HIPCHECK(node(R.maxOverflowDate, S.maxOverflowDate));
    HIPCHECK(node(R.maxPondedVol, S.maxPonded));
    HIPCHECK(nodeI(R.nonConvergedCount, S.nonConv));
    HIPCHECK(node(R.nodeInflowVol, S.mbIn));
    HIPCHECK(node(R.nodeOutflowVol, S.mbOut));
    HIPCHECK(node(R.outfallAvgFlow, S.oAvgFlow));
    HIPCHECK(node(R.outfallMaxFlow, S.oMaxFlow));
    HIPCHECK(nodeI(R.outfallPeriods, S.oPeriods));
    HIPCHECK(node(R.stAvgVol, S.sAvgVol));
    HIPCHECK(node(R.stMaxVol, S.sMaxVol));
    HIPCHECK(node(R.stMaxVolDate, S.sMaxVolDate));
    HIPCHECK(node(R.stMaxFlow, S.sMaxFlow));
    HIPCHECK(node(R.stEvapLoss, S.sEvap));
    HIPCHECK(node(R.stExfilLoss, S.sExfil));
    {
        size_t P = p.P;
        R.outfallLoad.assign(P * gN, 0.0);
        if (P) {
            tmp.resize(P * nN);
            HIPCHECK(hipMemcpy(tmp.data(), S.oLoad, P * nN * sizeof(double), hipMemcpyDeviceToHost));
            for (size_t q = 0; q < P; q++)
                for (size_t i = 0; i < nN; i++)
                    if (!multi || part.owned[i]) R.outfallLoad[q * gN + (multi ? part.lnode[i] : i)] = tmp[q * nN + i];
        }
    }
    HIPCHECK(link(R.lMaxFlow, S.lMaxFlow, 1));
    HIPCHECK(link(R.lMaxFlowDate, S.lMaxFlowDate, 1));
    HIPCHECK(link(R.lMaxVeloc, S.lMaxVeloc, 1));
    HIPCHECK(link(R.lMaxDepth, S.lMaxDepth, 1));
    HIPCHECK(link(R.lTimeNormalFlow, S.lTimeNormal, 1));
    HIPCHECK(link(R.lTimeInletControl, S.lTimeInlet, 1));
    HIPCHECK(link(R.lTimeSurcharged, S.lTimeSurch, 1));
    HIPCHECK(link(R.lTimeFullUpstream, S.lTimeFullUp, 1));
    HIPCHECK(link(R.lTimeFullDnstream, S.lTimeFullDn, 1));
    HIPCHECK(link(R.lTimeFullFlow, S.lTimeFullFlow, 1));
    HIPCHECK(link(R.lTimeCapacityLimited, S.lTimeCapLim, 1));
    HIPCHECK(link(R.lTimeInFlowClass, S.lTimeClass, RunStats::kClasses));
    HIPCHECK(link(R.lTimeCourantCritical, S.lTimeCourant, 1));
    HIPCHECK(linkI(R.lFlowTurns, S.lTurns));
    HIPCHECK(link(R.pUtilized, p.pUtil, 1));
    HIPCHECK(link(R.pMinFlow, p.pMin, 1));
    HIPCHECK(link(R.pAvgFlow, p.pAvg, 1));
    HIPCHECK(link(R.pMaxFlow, p.pMax, 1));
    HIPCHECK(link(R.pVolume, p.pVol, 1));
    HIPCHECK(link(R.pEnergy, p.pEnergy, 1));
    HIPCHECK(link(R.pOffLow, p.pOffLow, 1));
    HIPCHECK(link(R.pOffHigh, p.pOffHigh, 1));
    HIPCHECK(linkI(R.pStartUps, p.pStarts));
    HIPCHECK(linkI(R.pPeriods, p.pPeriods));
    HIPCHECK(linkI(R.lFlowTurnSign, S.lTurnSign));
    HIPCHECK(hipMemcpy(d->hostCtl, d->ctl, sizeof(StepCtl), hipMemcpyDeviceToHost));
    const StepCtl* c = d->hostCtl;
    R.reportStepCount = (double)c->reportStepCount;
    R.routingTimeSpan = c->routingTimeSpan;
    R.maxOutfallFlow = c->maxOutfallFlow;
    R.minTimeStep = c->tsMin;
    R.maxTimeStep = c->tsMax;
    R.routingTime = c->tsRoutingTime;
    R.steadyStateTime = c->tsSteadyTime;
    R.timeStepCount = (double)c->tsCount;
    R.trialsCount = (double)c->tsTrials;
    for (int j = 0; j < RunStats::kLevels; j++) {
        R.timeStepCounts[j] = (double)c->tsCounts[j];
        R.timeStepIntervals[j] = c->tsIntervals[j];
    }
    if (R.maxRptDepth.size() != gN) R.maxRptDepth.assign(gN, 0.0);   // host side (saveResults)
    R.valid = true;
    return 0;
}

int Router::upload(Project& prj)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    Params& p = d->p;
    State& st = prj.st;
    const Partition& part = d->part;
    const bool multi = part.active();
    size_t nN = p.nN, nL = p.nL;
    // stage buffers live until the final synchronize
    std::vector<std::vector<double>> stage;
    auto upN = [&](double* dst, const std::vector<double>& v) {
        if (!multi) return hipMemcpyAsync(dst, v.data(), nN * sizeof(double), hipMemcpyHostToDevice, d->stream);
        // replicas keep their device values (their owner's mirror is elsewhere)
        stage.emplace_back(nN);
        hipError_t r = hipMemcpy(stage.back().data(), dst, nN * sizeof(double), hipMemcpyDeviceToHost);
        if (r != hipSuccess) return r;
        for (size_t i = 0; i < nN; i++)
            if (part.owned[i]) stage.back()[i] = v[part.lnode[i]];
        return hipMemcpyAsync(dst, stage.back().data(), nN * sizeof(double), hipMemcpyHostToDevice, d->stream);
    };
    auto upL = [&](double* dst, const std::vector<double>& v) {
        if (!multi) return hipMemcpyAsync(dst, v.data(), nL * sizeof(double), hipMemcpyHostToDevice, d->stream);
        stage.emplace_back(nL);
        for (size_t j = 0; j < nL; j++) stage.back()[j] = v[part.llink[j]];
        return hipMemcpyAsync(dst, stage.back().data(), nL * sizeof(double), hipMemcpyHostToDevice, d->stream);
    };
    stage.reserve(16);
    HIPCHECK(upN(p.nNewDepth, st.newDepth));
    HIPCHECK(upN(p.nOldDepth, st.oldDepth));
    HIPCHECK(upN(p.nNewVolume, st.newVolume));
    HIPCHECK(upN(p.inflow, st.inflow));
    HIPCHECK(upN(p.outflow, st.outflow));
    HIPCHECK(upN(p.newLat, st.newLatFlow));
    if (st.hrt.size() == (size_t)prj.net.nNodes()) HIPCHECK(upN(p.hrt, st.hrt));
    HIPCHECK(upL(p.lNewFlow, st.lNewFlow));
    HIPCHECK(upL(p.lNewDepth, st.lNewDepth));
    HIPCHECK(upL(p.lNewVolume, st.lNewVolume));
    HIPCHECK(upL(p.q1, st.q1));
    HIPCHECK(upL(p.a1, st.a1));
    HIPCHECK(upL(p.setting, st.setting));
    WAITCHECK(waitDone(d_, nullptr));
    return 0;
}

// copy the device step clock/accounting block to its pinned host mirror;
// a failure (e.g. a faulted kernel) is latched into the router's error state
static void pullCtl(Router::Impl* d, int& err, std::string& msg)
{
    hipError_t e = hipMemcpyAsync(d->hostCtl, d->ctl, sizeof(StepCtl), hipMemcpyDeviceToHost,
                                  d->stream);
    if (e == hipSuccess && waitDone(d, nullptr) && !err) {
        err = 500;
        msg = "ERROR 500: GPU router: " + d->xerrMsg;
    }
    if (e != hipSuccess && !err) {
        err = 500;
        msg = std::string("ERROR 500: GPU router: ") + hipGetErrorString(e);
    }
    if (e == hipSuccess && d->hostCtl->tailErr && !err) {
        err = 500;
        msg = "ERROR 500: GPU router: k_tail grid barrier timed out (workgroups not co-resident)";
    }
}

void Router::counters(long long* totalIters, long long* nonConv, int* lastSteps)
{
    Impl* d = d_;
    pullCtl(d, err_, errMsg_);
    *totalIters = d->hostCtl->totalIters;
    *nonConv = d->hostCtl->nonConverge;
    *lastSteps = d->hostCtl->lastSteps;
}

void Router::flowTotals(double out[8])
{
    Impl* d = d_;
    pullCtl(d, err_, errMsg_);
    for (int q = 0; q < 8; q++) out[q] = d->hostCtl->flowTot[q];
}

void Router::stepTotals(double out[6])
{
    Impl* d = d_;
    pullCtl(d, err_, errMsg_);
    for (int q = 0; q < 6; q++) out[q] = d->hostCtl->prevStepTot[q];
}

void Router::setTiming(bool on)
{
    flushTiming(d_);
    if (!d_->probeSum.empty()) {                   // SWMM5_PROBE report (stderr)
        const int C = kProbeSlots + 7;
        fprintf(stderr, "probe (us after the first link workgroup start): k n  link_last_start  link_end  link_work_end  node_start  node_last_start  prologue_end  node_end  node_block0_end | node workgroup duration median max (slowest workgroup) | outfall tables_staged ynorm_done ycrit_done | link workgroup median scan staged walked\n");
        for (int k = 0; k * C < (int)d_->probeSum.size(); k++) {
            const double* o = d_->probeSum.data() + (size_t)C * k;
            if (o[kProbeSlots] <= 0) continue;
            const double n = o[kProbeSlots];
            fprintf(stderr, "probe k=%d n=%.0f  %.2f  %.2f  %.2f  %.2f  %.2f  %.2f  %.2f  %.2f | %.2f %.2f (%.0f) | %.2f %.2f %.2f | %.2f %.2f %.2f\n",
                    k, n, o[PR_L_IN] / n, o[PR_L_OUT] / n, o[PR_L_WORK] / n, o[PR_N_IN] / n, o[PR_N_LAST_IN] / n,
                    o[PR_N_PRO] / n, o[PR_N_OUT] / n, o[PR_N_B0] / n, o[kProbeSlots + 1] / n, o[kProbeSlots + 2] / n,
                    o[kProbeSlots + 3], o[PR_P_STAGED] / n, o[PR_P_YN] / n, o[PR_P_YC] / n, o[kProbeSlots + 4] / n,
                    o[kProbeSlots + 5] / n, o[kProbeSlots + 6] / n);
        }
        d_->probeSum.clear();
    }
    if (on && getenv("SWMM5_PROBE") && !d_->p.probe) {
        const int B = std::max(std::max(std::max(d_->gridL, d_->gridN), d_->gridLinkSparse), d_->gridNList);
        const size_t n = (size_t)std::max(d_->p.maxTrials, 1) * kProbeSlots * B;
        if (hipMalloc((void**)&d_->p.probe, n * sizeof(unsigned long long)) == hipSuccess &&
            hipMemset(d_->p.probe, 0, n * sizeof(unsigned long long)) == hipSuccess)
            d_->p.probeBlocks = B;
        else
            d_->p.probe = nullptr;
    } else if (!on && d_->p.probe) {
        (void)hipStreamSynchronize(d_->stream);
        (void)hipFree(d_->p.probe);
        d_->p.probe = nullptr;
        d_->p.probeBlocks = 0;
    }
    d_->timing = on;
    if (!on) d_->curX = nullptr;
    if (on && d_->p.nodeWork) {                    // the per-node work of the steps timed from now on
        (void)hipMemsetAsync(d_->p.nodeWork, 0, std::max<size_t>(d_->p.nN, 1) * sizeof(unsigned), d_->stream);
        (void)hipMemsetAsync(d_->p.nodeLinkWork, 0, std::max<size_t>(d_->p.nN, 1) * sizeof(unsigned), d_->stream);
    }
    d_->p.countWork = on ? 1 : 0;                  // eager launches only; the graph keeps 0
    for (int k = 0; k < Impl::kClasses; k++) { d_->kms[k] = 0; d_->kcnt[k] = 0; d_->kbytesSum[k] = 0; }
    d_->workSum = 0;
    d_->itersTimed1 = 0;
    d_->iterStats.clear();
    d_->gatherSum = 0;
    d_->gatherCnt = 0;
}

// Back-to-back replays of one kernel between two events (average duration per
// launch, dispatch gaps amortised).  The kernels run on the live state; this
// is a measurement tool (bench.py calls it after the timed run).
int Router::timeKernel(int which, int reps, double* avgUs)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    Params p = d->p;
    p.countWork = 0;
    hipEvent_t a, b;
    HIPCHECK(hipEventCreate(&a));
    HIPCHECK(hipEventCreate(&b));
    WAITCHECK(waitDone(d_, nullptr));
    HIPCHECK(hipEventRecord(a, d->stream));
    // the probe instantiations (distinct kernel names, same code)
    LinkKernelFn lk = nullptr;
    switch (d->linkWaves) {
    case 3: lk = d->fastLinks ? k_link<true, 3, true, true> : k_link<true, 3, false, true>; break;
    case 4: lk = d->fastLinks ? k_link<true, 4, true, true> : k_link<true, 4, false, true>; break;
    default: lk = d->fastLinks ? k_link<true, 1, true, true> : k_link<true, 1, false, true>; break;
    }
    LinkKernelFn nk = d->general ? k_node<true, true, true> : k_node<true, false, true>;
    for (int r = 0; r < reps; r++) {
        if (which == 0)
            hipLaunchKernelGGL(lk, dim3(d->gridL), dim3(kBlock), 0, d->stream, p, 0);
        else
            hipLaunchKernelGGL(nk, dim3(d->gridN), dim3(kBlock), 0, d->stream, p, 0);
    }
    HIPCHECK(hipEventRecord(b, d->stream));
    HIPCHECK(hipEventSynchronize(b));
    float ms = 0;
    HIPCHECK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *avgUs = 1000.0 * ms / std::max(reps, 1);
    return 0;
}

// ---- fine-grained state access (swmm_getValue / swmm_setValue) ----------
static int localIndex(const std::vector<int>& g2l, bool multi, int g)
{
    if (!multi) return g;
    return (g >= 0 && g < (int)g2l.size()) ? g2l[g] : -1;
}

int Router::peek(int field, int g, double* v)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    const Params& p = d->p;
    const bool multi = d->part.active();
    const double* src = nullptr;
    int i = -1;
    if (field < PK_LINK_FLOW) {
        i = localIndex(d->part.gnode, multi, g);
        if (i < 0 || i >= p.nN) return 1;
        switch (field) {
        case PK_NODE_DEPTH: src = p.nNewDepth; break;
        case PK_NODE_VOLUME: src = p.nNewVolume; break;
        case PK_NODE_LATFLOW: src = p.newLat; break;
        case PK_NODE_INFLOW: src = p.inflow; break;
        case PK_NODE_OVERFLOW: src = p.overflow; break;
        default: return 1;
        }
    } else {
        i = localIndex(d->part.glink, multi, g);
        if (i < 0 || i >= p.nL) return 1;
        switch (field) {
        case PK_LINK_FLOW: src = p.lNewFlow; break;
        case PK_LINK_DEPTH: src = p.lNewDepth; break;
        case PK_LINK_SETTING: src = p.setting; break;
        default: return 1;
        }
    }
    HIPCHECK(hipMemcpyAsync(v, src + i, sizeof(double), hipMemcpyDeviceToHost, d->stream));
    WAITCHECK(waitDone(d_, nullptr));
    return 0;
}

int Router::setOutfallStage(int g, double stage)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    Params& p = d->p;
    int i = localIndex(d->part.gnode, d->part.active(), g);
    if (i < 0 || i >= p.nN) return 0;                   // not on this rank
    WAITCHECK(waitDone(d_, nullptr));
    int f = 0;
    HIPCHECK(hipMemcpy(&f, p.nflags + i, sizeof(int), hipMemcpyDeviceToHost));
    f = (int)(((uint32_t)f & ~(0x7u << NF_OTYPE_SHIFT)) | ((uint32_t)O_FIXED << NF_OTYPE_SHIFT));
    HIPCHECK(hipMemcpy((void*)(p.nflags + i), &f, sizeof(int), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy((void*)(p.fixedStage + i), &stage, sizeof(double), hipMemcpyHostToDevice));
    return 0;
}

// swmm_stride (swmm5.c:466-510) ends the routing period at the stride's end
// and lowers RouteStep to the stride for the steps it runs, then restores
// both.  The reference takes each step's length at the start of that step
// (routing_getRoutingStep(RouteStep), counting the Courant-critical element
// if the step is routed at all); the engine chose the pending step's length
// at the end of the previous one, under the cap and period end then in force
// (durBefore).  It is chosen again here under `cap` and durAfter from the
// same uncapped Courant minima (StepCtl::stepRed), the critical-element count
// moved with it, and the end of the period re-applied.
int Router::repickStep(double cap, double durBefore, double durAfter)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    const Params& p = d->p;
    WAITCHECK(waitDone(d_, nullptr));
    HIPCHECK(hipMemcpy(d->hostCtl, d->ctl, sizeof(StepCtl), hipMemcpyDeviceToHost));
    StepCtl* h = d->hostCtl;
    const double oldCap = h->routeStep;
    h->routeStep = cap;
    h->routingDuration = durAfter;
    if (!p.varStep || h->varStepOff) {
        h->dtNext = cap;                                   // fixed step
    } else if (h->totalSteps > 0) {                        // the first step is MinRouteStep whatever the cap
        int c0 = 0, c1 = 0;
        (void)courantStep(h->stepRed[5], h->stepRed[6], oldCap, p.minRouteStep, &c0);
        const double t = courantStep(h->stepRed[5], h->stepRed[6], cap, p.minRouteStep, &c1);
        if (!(h->newRoutingTime < durBefore)) c0 = 0;     // k_finalize did not count it
        if (!(h->newRoutingTime < durAfter)) c1 = 0;      // the reference will not
        if (c0 != c1 && !p.multi) {
            auto bump = [&](int crit, double by) -> int {
                double* a = (crit == 2) ? p.st.timeCourant + (int)h->stepRed[9]
                                        : p.st.lTimeCourant + (int)h->stepRed[8];
                double v = 0.0;
                HIPCHECK(hipMemcpy(&v, a, sizeof(double), hipMemcpyDeviceToHost));
                v += by;
                HIPCHECK(hipMemcpy(a, &v, sizeof(double), hipMemcpyHostToDevice));
                return 0;
            };
            if (c0 && bump(c0, -1.0)) return err_;
            if (c1 && bump(c1, 1.0)) return err_;
        }
        h->variableStep = t;
        h->dtNext = t;
    }
    double dtn = h->dtNext > 0 ? h->dtNext : h->dt;
    if (h->newRoutingTime + 1000.0 * dtn > durAfter) {
        dtn = (durAfter - h->newRoutingTime) / 1000.0;
        dtn = (dtn >= 1. / 1000.0) ? dtn : 1. / 1000.0;
    }
    h->dt = dtn;
    HIPCHECK(hipMemcpy(d->ctl, d->hostCtl, sizeof(StepCtl), hipMemcpyHostToDevice));
    d->hostDt[d->launched % Impl::kRing] = dtn;            // the next step's slot
    return 0;
}

// climate_setState's evaporation rate for the next step; uploaded only when it
// changes (a month boundary or a time-series entry), behind the queued steps
int Router::setClimate(double rate, double hydcon, double recovery)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    const double v[3] = {rate, hydcon, recovery};
    if (v[0] == d->climateDev[0] && v[1] == d->climateDev[1] && v[2] == d->climateDev[2]) return 0;
    // in stream order ahead of the next step, from a pinned ring slot (a
    // time-series rate with an adjustment changes every step: no sync)
    if (!d->evapPinned) {
        HIPCHECK(hipHostMalloc((void**)&d->evapPinned, 3 * Impl::kRing * sizeof(double), hipHostMallocDefault));
        for (auto& ev : d->evapEv) {
            HIPCHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            HIPCHECK(hipEventRecord(ev, d->stream));
        }
    }
    const int sl = d->evapNext;
    d->evapNext = (d->evapNext + 1) % Impl::kRing;
    WAITCHECK(waitDone(d_, d->evapEv[sl]));           // the copy that last read this slot
    double* slot = d->evapPinned + 3 * sl;
    for (int q = 0; q < 3; q++) slot[q] = v[q];
    static_assert(offsetof(StepCtl, hydconFactor) == offsetof(StepCtl, evapRate) + sizeof(double) &&
                  offsetof(StepCtl, recoveryFactor) == offsetof(StepCtl, evapRate) + 2 * sizeof(double),
                  "the climate values are copied as one block");
    HIPCHECK(hipMemcpyAsync(&d->p.ctl->evapRate, slot, 3 * sizeof(double), hipMemcpyHostToDevice, d->stream));
    HIPCHECK(hipEventRecord(d->evapEv[sl], d->stream));
    for (int q = 0; q < 3; q++) d->climateDev[q] = v[q];
    return 0;
}

int Router::setRouteStep(double step, double dtNext)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    WAITCHECK(waitDone(d_, nullptr));
    StepCtl* c = d->p.ctl;
    int off = 1;
    HIPCHECK(hipMemcpy(&c->routeStep, &step, sizeof(double), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(&c->varStepOff, &off, sizeof(int), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(&c->dt, &dtNext, sizeof(double), hipMemcpyHostToDevice));
    return 0;
}

// k_pack_results into d->resN / d->resL (allocated on first use), on the stream
static int launchPack(Router::Impl* d, double f, double uL, double uV, double uQ, std::string* msg)
{
    const Params& p = d->p;
    size_t nb = (size_t)p.nN * (6 + p.P), lb = (size_t)p.nL * (5 + p.P);
    hipError_t e = hipSuccess;
    if (!d->resN) {
        d->resN = devAlloc<float>(d, nb, &e);
        if (e == hipSuccess) d->resL = devAlloc<float>(d, lb, &e);
        if (e == hipSuccess) e = hipHostMalloc((void**)&d->resNHost, std::max<size_t>(nb, 1) * sizeof(float), hipHostMallocDefault);
        if (e == hipSuccess) e = hipHostMalloc((void**)&d->resLHost, std::max<size_t>(lb, 1) * sizeof(float), hipHostMallocDefault);
        if (e != hipSuccess) { *msg = hipGetErrorString(e); return 1; }
    }
    int grid = std::max(d->gridL, d->gridN);
    if (d->fastLinks)
        hipLaunchKernelGGL(k_pack_results<true>, dim3(grid), dim3(kBlock), 0, d->stream, p, f, uL, uV, uQ,
                           d->resN, d->resL);
    else
        hipLaunchKernelGGL(k_pack_results<false>, dim3(grid), dim3(kBlock), 0, d->stream, p, f, uL, uV, uQ,
                           d->resN, d->resL);
    e = hipGetLastError();
    if (e != hipSuccess) { *msg = hipGetErrorString(e); return 1; }
    return 0;
}

int Router::avgUpdate(double uL, double uV, double uQ)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    const Params& p = d->p;
    size_t nb = (size_t)p.nN * (6 + p.P), lb = (size_t)p.nL * (5 + p.P);
    std::string m;
    if (launchPack(d, 1.0, uL, uV, uQ, &m)) { fail(m); return err_; }
    if (!d->avgN) {
        hipError_t e;
        d->avgN = devAlloc<float>(d, nb, &e);
        if (e == hipSuccess) d->avgL = devAlloc<float>(d, lb, &e);
        if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
        HIPCHECK(hipMemsetAsync(d->avgN, 0, std::max<size_t>(nb, 1) * sizeof(float), d->stream));
        HIPCHECK(hipMemsetAsync(d->avgL, 0, std::max<size_t>(lb, 1) * sizeof(float), d->stream));
    }
    int grid = std::max(d->gridL, d->gridN);
    hipLaunchKernelGGL(k_avg_accum, dim3(grid), dim3(kBlock), 0, d->stream, p, d->resN, d->resL, d->avgN, d->avgL,
                       (float)(d->avgSteps + 1));
    HIPCHECK(hipGetLastError());
    d->avgSteps++;
    return 0;
}

int Router::avgTake(double uL, double uV, double uQ, const float** avgNode, const float** avgLink,
                    const float** curNode, const float** curLink, const double** depth)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    const Params& p = d->p;
    size_t nb = (size_t)p.nN * (6 + p.P), lb = (size_t)p.nL * (5 + p.P);
    std::string m;
    if (launchPack(d, 1.0, uL, uV, uQ, &m)) { fail(m); return err_; }
    if (!d->avgON) {
        hipError_t e;
        if (!d->avgN) {
            d->avgN = devAlloc<float>(d, nb, &e);
            if (e == hipSuccess) d->avgL = devAlloc<float>(d, lb, &e);
            if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
            HIPCHECK(hipMemsetAsync(d->avgN, 0, std::max<size_t>(nb, 1) * sizeof(float), d->stream));
            HIPCHECK(hipMemsetAsync(d->avgL, 0, std::max<size_t>(lb, 1) * sizeof(float), d->stream));
        }
        d->avgON = devAlloc<float>(d, nb, &e);
        if (e == hipSuccess) d->avgOL = devAlloc<float>(d, lb, &e);
        if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
        HIPCHECK(hipHostMalloc((void**)&d->avgONHost, std::max<size_t>(nb, 1) * sizeof(float), hipHostMallocDefault));
        HIPCHECK(hipHostMalloc((void**)&d->avgOLHost, std::max<size_t>(lb, 1) * sizeof(float), hipHostMallocDefault));
        HIPCHECK(hipHostMalloc((void**)&d->depthHost, std::max<int>(p.nN, 1) * sizeof(double), hipHostMallocDefault));
    }
    int grid = std::max(d->gridL, d->gridN);
    hipLaunchKernelGGL(k_avg_take, dim3(grid), dim3(kBlock), 0, d->stream, nb, lb, d->avgN, d->avgL, d->avgON,
                       d->avgOL, (float)d->avgSteps);
    HIPCHECK(hipGetLastError());
    d->avgSteps = 0;
    HIPCHECK(hipMemcpyAsync(d->avgONHost, d->avgON, nb * sizeof(float), hipMemcpyDeviceToHost, d->stream));
    HIPCHECK(hipMemcpyAsync(d->avgOLHost, d->avgOL, lb * sizeof(float), hipMemcpyDeviceToHost, d->stream));
    HIPCHECK(hipMemcpyAsync(d->resNHost, d->resN, nb * sizeof(float), hipMemcpyDeviceToHost, d->stream));
    HIPCHECK(hipMemcpyAsync(d->resLHost, d->resL, lb * sizeof(float), hipMemcpyDeviceToHost, d->stream));
    HIPCHECK(hipMemcpyAsync(d->depthHost, p.nNewDepth, (size_t)p.nN * sizeof(double), hipMemcpyDeviceToHost,
                            d->stream));
    WAITCHECK(waitDone(d_, nullptr));
    *avgNode = d->avgONHost;
    *avgLink = d->avgOLHost;
    *curNode = d->resNHost;
    *curLink = d->resLHost;
    *depth = d->depthHost;
    return 0;
}

int Router::packResults(double f, double uL, double uV, double uQ, const float** nodeVals,
                        const float** linkVals)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    const Params& p = d->p;
    size_t nb = (size_t)p.nN * (6 + p.P), lb = (size_t)p.nL * (5 + p.P);
    std::string m;
    if (launchPack(d, f, uL, uV, uQ, &m)) { fail(m); return err_; }
    HIPCHECK(hipMemcpyAsync(d->resNHost, d->resN, nb * sizeof(float), hipMemcpyDeviceToHost, d->stream));
    HIPCHECK(hipMemcpyAsync(d->resLHost, d->resL, lb * sizeof(float), hipMemcpyDeviceToHost, d->stream));
    WAITCHECK(waitDone(d_, nullptr));
    *nodeVals = d->resNHost;
    *linkVals = d->resLHost;
    return 0;
}

const Partition& Router::partition() const { return d_->part; }

int Router::nodeWork(double* out, int n, bool conduits)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    flushTiming(d);
    std::vector<unsigned> w((size_t)std::max(d->p.nN, 1));
    WAITCHECK(waitDone(d_, nullptr));
    HIPCHECK(hipMemcpy(w.data(), conduits ? d->p.nodeLinkWork : d->p.nodeWork, w.size() * sizeof(unsigned),
                       hipMemcpyDeviceToHost));
    const Partition& part = d->part;
    for (int i = 0; i < d->p.nN; i++) {
        const int g = part.active() ? part.lnode[i] : i;
        if (g < n && (!part.active() || part.owned[i])) out[g] = (double)w[i];
    }
    return 0;
}
std::string Router::transport() const { return d_->transportName; }

int Router::allreduceHost(double* buf, int n, int op)
{
    auto fail = [&](const std::string& m) { err_ = 500; errMsg_ = "ERROR 500: GPU router: " + m; };
    Impl* d = d_;
    if (!d->part.active() || n <= 0) return 0;
    // the host callback when one is set (host transport; IPC bootstrapped over
    // it), else the RCCL communicator
    if (d->part.xchg) {
        if (d->part.xchg(buf, n, op, d->part.xuser)) { fail("host exchange failed"); return err_; }
        return 0;
    }
    if (!d->comm) { fail("no communicator (aborted after an earlier failure)"); return err_; }
    double* tmp = nullptr;
    HIPCHECK(hipMalloc(&tmp, n * sizeof(double)));
    hipError_t e = hipMemcpyAsync(tmp, buf, n * sizeof(double), hipMemcpyHostToDevice, d->stream);
    if (e == hipSuccess) {
        ncclResult_t r = ncclAllReduce(tmp, tmp, n, ncclDouble, op ? ncclMin : ncclSum, d->comm, d->stream);
        if (r != ncclSuccess) { (void)hipFree(tmp); fail(std::string("ncclAllReduce: ") + ncclGetErrorString(r)); return err_; }
        e = hipMemcpyAsync(buf, tmp, n * sizeof(double), hipMemcpyDeviceToHost, d->stream);
    }
    if (e == hipSuccess && waitDone(d, nullptr)) {
        (void)hipFree(tmp);
        fail(d->xerrMsg);
        return err_;
    }
    (void)hipFree(tmp);
    if (e != hipSuccess) { fail(hipGetErrorString(e)); return err_; }
    return 0;
}

void Router::timedWork(double* updated, double* hot, double* gathered, double* gatherIters)
{
    flushTiming(d_);
    *updated = d_->workSum;
    *hot = d_->nHot;
    *gathered = d_->gatherSum;
    *gatherIters = d_->gatherCnt;
}

void Router::graphStats(long long out[9])
{
    flushTiming(d_);
    out[0] = d_->itersTimed1;
    for (int m = 0; m < 4; m++) out[1 + m] = d_->modeSteps[m];
    out[5] = d_->p.deferPro;
    out[6] = 0;                                    // retired counters (fused / compact graphs)
    out[7] = 0;
    out[8] = 0;
}

int Router::kernelTimes(double* out, int n)
{
    flushTiming(d_);
    int m = std::min(n / 2, (int)Impl::kClasses);
    for (int k = 0; k < m; k++) {
        out[2 * k] = (double)d_->kcnt[k];
        out[2 * k + 1] = d_->kms[k];
    }
    return m;
}

int Router::iterationStats(double* out, int n)
{
    flushTiming(d_);
    const int m = std::min(n, (int)d_->iterStats.size());
    for (int k = 0; k < m; k++) out[k] = d_->iterStats[k];
    return (int)d_->iterStats.size();
}

int Router::kernelBytes(double* out, int n)
{
    flushTiming(d_);
    // average algorithmic bytes per timed launch (byte model when nothing was timed)
    int m = std::min(n, (int)Impl::kClasses);
    for (int k = 0; k < m; k++) {
        double model = (k == 4) ? d_->kbytes[4] * d_->nHot : d_->kbytes[k];
        out[k] = d_->kcnt[k] ? d_->kbytesSum[k] / (double)d_->kcnt[k] : model;
    }
    return m;
}

// ---------------------------------------------------------------------------
// Known-answer evaluation of the cross-section relations on the device
// (swmmx_xsect with device = 1): the same xsect.h code the kernels run, with
// the device's libm
__global__ void k_xsect_eval(Geom g, int fn, const double* x, double* y, int n, const double* circ)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = evalXsect(g, fn, x[i], circ);
}

int xsectEvalDevice(const Geom& gh, int fn, const double* x, double* y, int n)
{
    if (n <= 0) return 0;
    Geom g = gh;
    double *dx = nullptr, *dy = nullptr, *dc = nullptr, *ds = nullptr;
    size_t nb = (size_t)n * sizeof(double);
    bool ok = hipMalloc(&dx, nb) == hipSuccess && hipMalloc(&dy, nb) == hipSuccess &&
              hipMalloc(&dc, sizeof(double) * 5 * SWX_CIRC_N) == hipSuccess &&
              hipMalloc(&ds, sizeof(double) * SWX_SHAPE_TAB_LEN) == hipSuccess;
    if (ok) {
        (void)hipMemcpy(dx, x, nb, hipMemcpyHostToDevice);
        (void)hipMemcpy(dc, &SWX_CIRC_TABLES[0][0], sizeof(double) * 5 * SWX_CIRC_N, hipMemcpyHostToDevice);
        (void)hipMemcpy(ds, SWX_SHAPE_TAB, sizeof(double) * SWX_SHAPE_TAB_LEN, hipMemcpyHostToDevice);
        int off = shapeTabOffset(g.type);
        g.tb = (off >= 0) ? ds + off : nullptr;
        hipLaunchKernelGGL(k_xsect_eval, dim3((n + 255) / 256), dim3(256), 0, 0, g, fn, dx, dy, n, dc);
        ok = hipDeviceSynchronize() == hipSuccess &&
             hipMemcpy(y, dy, nb, hipMemcpyDeviceToHost) == hipSuccess;
    }
    (void)hipFree(dx); (void)hipFree(dy); (void)hipFree(dc); (void)hipFree(ds);
    return ok ? 0 : 500;
}

}  // namespace swx
