// router.h -- the HBM-resident dynamic-wave router (device side of the engine).
//
// Owns every device array (structure-of-arrays link/node state, the node->link
// CSR that reproduces the reference's serial summation order, the LDS-staged
// geometry tables) and one HIP stream.  A routing step is one replay of a
// captured HIP graph: MaxTrials x {link momentum, node update} kernel pairs with
// on-device early exit after convergence (no host round trip inside the Picard
// loop), then the step-end accounting kernels.  See DESIGN.md.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "partition.h"
#include "project.h"

namespace swx {

struct RouterTotals {            // system flow totals kept on the device (massbal.c)
    double dwInflow, exInflow, flooding, outflow, evapLoss, seepLoss;  // volumes (ft3)
    double initStorage;
};

class Router {
public:
    Router();
    ~Router();
    // Allocate + upload static network and initial state; build graph.  With
    // a multi-rank partition only this rank's part of the network is uploaded
    // and every Picard iteration all-reduces the shared-node sums.
    int init(Project& prj, int device, const Partition* part = nullptr);
    // Enqueue one routing step.  The step length and the simulation clock
    // live on the device (k_finalize computes the next dt exactly as
    // dynwave_getRoutingStep + execRouting's clamp do), so a fixed-step run
    // never synchronises.  latFlow/qualLoad: this step's lateral flows / mass
    // loads (nullptr = the constant arrays evaluated at init); totals =
    // {dwInflow, exInflow, exOutflow} rates of those inflows.
    int step(const double* latFlow, const double* qualLoad, const double totals[3]);
    // dt (sec) of the step most recently passed to step(); waits only for the
    // previous step to finish, so one step stays queued on the device
    int launchedDt(double* dt);
    // Read the device clock after the last enqueued step (synchronises):
    // routing time (msec) and the step length used by that step.
    int readClock(double* newRoutingTime, double* lastDt, double* nextDt);
    // conduits updated by the timed iterations >= 1, and streaming conduits
    void timedWork(double* updated, double* hot, double* gathered, double* gatherIters);
    // timed iterations k >= 1 that ran; steps launched with the unrolled,
    // k_tail, k_sparse and list step graphs
    void graphStats(long long out[9]);   // timed iterations, steps per graph, deferred outfalls, compact growth
    // Sum (op 0) or min (op 1) of n host doubles over the ranks (no-op on one GPU).
    int allreduceHost(double* buf, int n, int op);
    // average duration (us) of `reps` back-to-back launches of kernel `which`
    // (0 k_link<first>, 1 k_node<first>) on the live state -- measurement only
    int timeKernel(int which, int reps, double* avgUs);
    // this rank's partition (whole network when running on one GPU)
    const Partition& partition() const;
    // Change the routing duration (msec) used for the end-of-run clamp.
    // Copy device state into the host mirror (prj.st); synchronises.
    int download(Project& prj);
    // One state value of node / link g (global index) straight from HBM;
    // returns nonzero when the object is not held by this rank.  Synchronises.
    enum { PK_NODE_DEPTH, PK_NODE_VOLUME, PK_NODE_LATFLOW, PK_NODE_INFLOW, PK_NODE_OVERFLOW,
           PK_LINK_FLOW, PK_LINK_DEPTH, PK_LINK_SETTING };
    int peek(int field, int g, double* v);
    // swmm_setValue(NODE_HEAD) on an outfall: FIXED type with this stage (ft)
    // (setOutfallStage, swmm5.c:1173-1188)
    int setOutfallStage(int g, double stage);
    // climate_setState's Evap.rate (ft/s), Adjust.hydconFactor and
    // Evap.recoveryFactor for the steps launched from now on
    int setClimate(double evapRate, double hydconFactor, double recoveryFactor);
    // swmm_setValue(ROUTESTEP) between steps (setRoutingStep, swmm5.c:1360-
    // 1370): fixed steps of `step` sec from now on, next step dtNext sec
    int setRouteStep(double step, double dtNext);
    // swmm_stride: routing-step cap and end of the routing period for the
    // following steps; the pending step's length is chosen again under them
    int repickStep(double cap, double durBefore, double durAfter);
    // Results of one reporting period packed on the device in the .out
    // variable order (nodes: 6 + P floats each, links: 5 + P), interpolated
    // with weight f and converted with the unit factors; pointers to pinned
    // host copies valid until the next call.  Synchronises.
    int packResults(double f, double uL, double uV, double uQ, const float** nodeVals,
                    const float** linkVals);
    // REPORT AVERAGES (output.c:857-955).  avgUpdate: add the current results
    // (packResults with f = 1) to the reporting period's float32 sums
    // (output_updateAvgResults).  avgTake: the period's averages, the current
    // results and the nodes' current depths (ft) on pinned host copies, then
    // the sums reset (output_saveAvgResults, output_initAvgResults).
    int avgUpdate(double uL, double uV, double uQ);
    int avgTake(double uL, double uV, double uQ, const float** avgNode, const float** avgLink,
                const float** curNode, const float** curLink, const double** depth);
    // Copy the run statistics accumulators into prj.stats; synchronises.
    int downloadStats(Project& prj);
    // Upload the host mirror's dynamic state (after swmm_setValue edits).
    int upload(Project& prj);
    int sync();
    // counters: total iterations, non-converging steps, iterations of last step
    void counters(long long* totalIters, long long* nonConv, int* lastSteps);
    void flowTotals(double out[8]);
    // system flow rates of the last completed step {dw, ex, flooding, outflow, evap, seep}
    void stepTotals(double out[6]);
    void setTiming(bool on);
    int kernelTimes(double* out, int n);
    int kernelBytes(double* out, int n);
    // per Picard iteration k of the timed steps, 7 values each: launches,
    // conduits updated, nodes gathered, nodes updated, relaxation-only node
    // updates, k_link ms, k_node ms; returns the number of values available
    int iterationStats(double* out, int n);
    // per global node (owned ones; out[] untouched elsewhere): its updates in
    // Picard iterations k >= 2 of the steps timed since setTiming(true), or
    // (conduits) the updates of the conduits it is node1 of (their owner
    // follows node1) in those iterations
    int nodeWork(double* out, int n, bool conduits = false);
    std::string deviceName() const { return devName_; }
    // the multi-GPU transport in use ("single", "rccl", "host", "ipc", or a
    // fallback note)
    std::string transport() const;
    bool ok() const { return ok_; }
    int lastError() const { return err_; }
    std::string lastErrorMsg() const { return errMsg_; }

    struct Impl;
private:
    Impl* d_;
    bool ok_ = false;
    int err_ = 0;
    std::string errMsg_, devName_;
};

// device evaluation of a cross-section relation (swmmx_xsect); 0 or 500
int xsectEvalDevice(const Geom& g, int fn, const double* x, double* y, int n);

}  // namespace swx
