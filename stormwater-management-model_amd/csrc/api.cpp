// api.cpp -- the C ABI (include/swmm5.h, include/swmm5_mi355x.h).
//
// Lifecycle and step driver restate the reference's supervisor
// (src/solver/swmm5.c): swmm_open 256-310, swmm_start 314-407, swmm_step
// 410-462 with execRouting 514-575 and saveResults 579-613, swmm_end 618-660,
// swmm_close 682-702, getters/setters 842-1213.  The routing itself is
// delegated to the HBM-resident Router (dw_kernels.hip); the host keeps a
// lazily synchronised mirror of the state for getValue, report-time output
// and the report file.  There is deliberately no CPU routing path: without a
// HIP device swmm_start fails with ERR_SYSTEM.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

#include <rccl/rccl.h>

#include "../../include/swmm5_mi355x.h"
#include "output.h"
#include "project.h"
#include "report.h"
#include "router.h"
#include "xsect.h"

using namespace swx;

namespace {

struct Engine {
    std::unique_ptr<Project> prj;
    std::unique_ptr<Router> router;
    OutFile out;
    std::string inpPath, rptPath, outPath;
    FILE* rpt = nullptr;
    bool isOpen = false, isStarted = false, hostOnly = false, saveFlag = true;
    bool mirrorValid = true;         // host mirror equals device state
    int errorCode = 0;
    bool stateSpent = false;        // swmmx_timeKernel replayed kernels on the live state
    std::string errorMsg;
    double newRoutingTime = 0.0, oldRoutingTime = 0.0, reportTime = 0.0;
    double routingDuration = 0.0, elapsedTime = 0.0;
    long long totalStepCount = 0;
    double flowError = 0.0, qualError = 0.0;
    double flowTot[8] = {0};
    double initStorage = 0.0, finalStorage = 0.0;
    double sysStep[6] = {0};
    double apiExtTouched = 0;
    std::vector<double> apiExtInflow;
    int device = -1;
    bool constantInflow = true;
};

Engine* G = nullptr;
int gDevice = -1;                    // swmmx_setDevice (survives swmm_open)
Partition gPart;                     // swmmx_setPartition / swmmx_setExchange (survive swmm_open)

int setErr(int code, const std::string& msg)
{
    if (G && !G->errorCode) {
        G->errorCode = code;
        G->errorMsg = msg;
        if (G->rpt) fprintf(G->rpt, "\n  %s\n", msg.c_str());
    }
    return code;
}

int syncMirror()
{
    if (!G || !G->router || G->mirrorValid) return 0;
    if (G->router->download(*G->prj)) return setErr(G->router->lastError(), G->router->lastErrorMsg());
    G->mirrorValid = true;
    return 0;
}

// Several GPUs: an error one rank alone met (rank 0 writes the results and
// hot start files) reaches every rank at the same point -- an all-reduce of
// the error codes (min of their negatives) -- so that no rank goes on into a
// collective the failed rank never reaches.  Called where such errors arise:
// the end of swmm_start, around each reporting period's gather, and in
// swmm_end before and after the hot start gather.  (A device failure inside a
// step is not covered: that would need an exchange every step.)
static int syncError()
{
    if (!G) return 501;
    if (!gPart.active()) return G->errorCode;
    double e = -(double)G->errorCode;
    // every rank joins, whatever its own state: over the host callback when
    // one is set (it needs no router), else over the router's communicator;
    // a rank with neither (RCCL before its communicator exists) cannot reach
    // the others
    if (gPart.xchg) {
        if (gPart.xchg(&e, 1, 1, gPart.xuser))
            return setErr(500, "ERROR 500: multi-GPU error exchange failed");
    } else if (G->router && G->router->ok()) {
        if (G->router->allreduceHost(&e, 1, 1)) return setErr(G->router->lastError(), G->router->lastErrorMsg());
    } else {
        return G->errorCode;
    }
    if (e < 0.0 && !G->errorCode)
        setErr((int)-e, "ERROR " + std::to_string((int)-e) + ": reported by another rank.");
    return G->errorCode;
}

int defaultDevice()
{
    const char* s = getenv("LOCAL_RANK");
    if (s) return atoi(s);
    return 0;
}

void writeReportHeader()
{
    if (!G->rpt) return;
    fprintf(G->rpt, "\n  EPA STORM WATER MANAGEMENT MODEL - VERSION 5.2 (Build 5.2.4)\n");
    fprintf(G->rpt, "  --------------------------------------------------------------\n");
    fprintf(G->rpt, "  MI355X dynamic-wave routing engine (libswmm5_mi355x)\n\n");
    if (!G->prj->net.title.empty()) fprintf(G->rpt, "  %s\n\n", G->prj->net.title.c_str());
}

}  // namespace

extern "C" {

int DLLEXPORT swmm_open(const char* f1, const char* f2, const char* f3)
{
    delete G;
    G = new Engine();
    G->prj.reset(new Project());
    if (!f1 || !f2 || !f3) return setErr(301, "ERROR 301: files share same names.");
    G->inpPath = f1; G->rptPath = f2; G->outPath = f3;
    if (!strcasecmp(f1, f2) || !strcasecmp(f1, f3) || !strcasecmp(f2, f3))
        return setErr(301, "ERROR 301: files share same names.");
    G->rpt = fopen(f2, "wt");
    if (!G->rpt) return setErr(305, "ERROR 305: cannot open report file.");
    G->isOpen = true;
    writeReportHeader();
    if (G->prj->open(f1)) {
        setErr(G->prj->errorCode, G->prj->errorMsg);
        // each further one, as report_writeErrorMsg (report.c:1422-1442):
        // written to the report; ErrorCode is the last code, ErrorMsg the last
        // message that is not about a line of input
        for (const auto& e : G->prj->moreErrors) {
            if (G->rpt) fprintf(G->rpt, "\n  %s\n", e.second.c_str());
            G->errorCode = e.first;
            if (e.first <= 200 || e.first >= 301) G->errorMsg = e.second;
        }
        return G->errorCode;
    }
    return G->errorCode;
}

int DLLEXPORT swmmx_startHost(void)
{
    if (!G) return 501;
    if (G->errorCode) return G->errorCode;
    if (!G->isOpen) return (G->errorCode = 501);
    if (G->isStarted) return (G->errorCode = 503);
    if (G->prj->initState()) return setErr(G->prj->errorCode, G->prj->errorMsg);
    G->hostOnly = true;
    G->isStarted = true;
    G->mirrorValid = true;
    return 0;
}

int DLLEXPORT swmm_start(int saveFlag)
{
    if (!G) return 501;
    if (G->errorCode) return G->errorCode;
    if (!G->isOpen) return (G->errorCode = 501);
    if (G->isStarted) return (G->errorCode = 503);
    Project& prj = *G->prj;
    G->saveFlag = saveFlag != 0;
    G->newRoutingTime = 0.0;
    G->oldRoutingTime = 0.0;
    G->reportTime = 1000.0 * (double)prj.opt.reportStep;
    G->routingDuration = prj.opt.totalDuration;
    G->totalStepCount = 0;
    G->elapsedTime = 0.0;
    // project_init, output_open and hotstart_open (swmm5.c:370-385); the
    // results file is opened first, as in the reference
    // (several GPUs: the results are gathered from the ranks that own them and
    // written by rank 0 alone, gatherResults; the other ranks write no file)
    const bool writer = !(gPart.active() && gPart.rank != 0);
    // (several GPUs: a failure to open the file is kept until every rank has
    // started its router, whose communicator the error exchange needs)
    bool openFailed = false;
    if (writer && G->out.open(G->outPath, prj)) {
        if (!gPart.active()) return setErr(307, "ERROR 307: cannot open binary results file.");
        openFailed = true;
    }
    if (prj.initState()) return setErr(prj.errorCode, prj.errorMsg);
    G->apiExtInflow.assign(prj.net.nNodes(), 0.0);
    G->constantInflow = prj.inflowsAreConstant();
    // massbal_open: initial storage
    double s = 0.0;
    for (int j = 0; j < prj.net.nNodes(); j++) s += prj.st.newVolume[j];
    for (int j = 0; j < prj.net.nLinks(); j++) s += prj.st.lNewVolume[j];
    G->initStorage = s;
    // StorageStats.initVol (stats.c:224)
    prj.stats.stInitVol.assign(prj.net.nNodes(), 0.0);
    for (int j = 0; j < prj.net.nNodes(); j++)
        if (prj.net.nodeType[j] == STORAGE) prj.stats.stInitVol[j] = prj.st.newVolume[j];
    G->router.reset(new Router());
    int dev = (gDevice >= 0) ? gDevice : defaultDevice();
    if (G->router->init(prj, dev, gPart.active() ? &gPart : nullptr)) {
        setErr(G->router->lastError(), G->router->lastErrorMsg());
        if (gPart.active()) syncError();            // the other ranks wait in the same exchange
        return G->errorCode;
    }
    if (openFailed) setErr(307, "ERROR 307: cannot open binary results file.");
    if (gPart.active() && syncError()) return G->errorCode;
    G->isStarted = true;
    G->mirrorValid = true;
    return G->errorCode;
}

static int execRouting()   // swmm5.c:514-575 + routing.c:203-265 on the device
{
    Project& prj = *G->prj;
    Router& r = *G->router;
    G->totalStepCount++;
    double currentDate = prj.getDateTime(G->newRoutingTime);
    // no runoff: climate_setState for evaporation (swmm5.c:555-556)
    const double evap = prj.climateSetState(currentDate);
    if (prj.errorCode) return setErr(prj.errorCode, prj.errorMsg);
    if (r.setClimate(evap, prj.opt.hydconFactor, prj.opt.recoveryFactor)) return setErr(r.lastError(), r.lastErrorMsg());
    int rc;
    if (G->constantInflow) {
        rc = r.step(nullptr, nullptr, nullptr);
    } else {
        std::vector<double> lat, qual;
        double tot[3];
        int P = prj.opt.ignoreQuality ? 0 : prj.net.nPollut();
        prj.evalInflows(currentDate, lat, P ? &qual : nullptr, &tot[0], &tot[1], &tot[2]);
        // apiExtInflow (swmm_setValue NODE_LATFLOW) is added by addExternalInflows
        for (int j = 0; j < prj.net.nNodes(); j++) {
            double q = G->apiExtInflow[j];
            if (q == 0.0) continue;
            if (fabs(q) < kFlowTol) q = 0.0;
            lat[j] += q;
            if (q >= 0.0) tot[1] += q; else tot[2] += -q;
        }
        rc = r.step(lat.data(), P ? qual.data() : nullptr, tot);
    }
    if (rc) return setErr(r.lastError(), r.lastErrorMsg());
    G->mirrorValid = false;
    // clock: identical arithmetic to the device's k_finalize (routing.c:301);
    // fixed steps are mirrored on the host, variable steps take the dt the
    // device chose at the end of the previous step (Router::launchedDt)
    G->oldRoutingTime = G->newRoutingTime;
    if (prj.opt.courantFactor == 0.0 || prj.opt.routeStep < 0.001) {
        double dt = prj.opt.routeStep;
        if (G->newRoutingTime + 1000.0 * dt > G->routingDuration) {
            dt = (G->routingDuration - G->newRoutingTime) / 1000.0;
            dt = (dt >= 1. / 1000.0) ? dt : 1. / 1000.0;
        }
        G->newRoutingTime = G->newRoutingTime + 1000.0 * dt;
    } else {
        double dt;
        if (r.launchedDt(&dt)) return setErr(r.lastError(), r.lastErrorMsg());
        G->newRoutingTime = G->newRoutingTime + 1000.0 * dt;
    }
    return 0;
}

// Several GPUs: the packed results of the objects each rank owns, in global
// object order, on every rank.  One all-reduce (min) over the ranks of
// arrays in which every slot another rank owns holds +inf: min(x, +inf) is x
// exactly (-0.0 included), so the gathered floats are the owners' bits.
// Segments: node rows (nv floats per node), link rows (lv per link), then
// with REPORT AVERAGES the averaged node and link rows and the node depths.
struct GatheredResults {
    std::vector<float> nv, lv, an, al;
    std::vector<double> depth;
};
static int gatherResults(const float* nv, const float* lv, const float* an, const float* al, const double* depth,
                         GatheredResults& g)
{
    const Partition& part = G->router->partition();
    const Network& net = G->prj->net;
    const size_t gN = net.nNodes(), gL = net.nLinks();
    const int P = G->prj->opt.ignoreQuality ? 0 : net.nPollut();
    const size_t nvv = 6 + P, lvv = 5 + P;
    const bool avg = an != nullptr;
    const size_t sN = gN * nvv, sL = gL * lvv;
    const size_t n = sN + sL + (avg ? sN + sL + gN : 0);
    std::vector<double> buf(n, INFINITY);
    for (size_t i = 0; i < part.lnode.size(); i++) {
        if (!part.owned[i]) continue;
        const size_t gi = part.lnode[i];
        for (size_t v = 0; v < nvv; v++) {
            buf[gi * nvv + v] = nv[i * nvv + v];
            if (avg) buf[sN + sL + gi * nvv + v] = an[i * nvv + v];
        }
        if (avg) buf[2 * (sN + sL) + gi] = depth[i];
    }
    for (size_t j = 0; j < part.llink.size(); j++) {
        const size_t gj = part.llink[j];
        for (size_t v = 0; v < lvv; v++) {
            buf[sN + gj * lvv + v] = lv[j * lvv + v];
            if (avg) buf[2 * sN + sL + gj * lvv + v] = al[j * lvv + v];
        }
    }
    if (n > (size_t)0x7FFFFFFF) return setErr(500, "ERROR 500: results too large to gather");
    if (G->router->allreduceHost(buf.data(), (int)n, 1)) return setErr(G->router->lastError(), G->router->lastErrorMsg());
    g.nv.assign(buf.begin(), buf.begin() + sN);
    g.lv.assign(buf.begin() + sN, buf.begin() + sN + sL);
    if (avg) {
        g.an.assign(buf.begin() + sN + sL, buf.begin() + 2 * sN + sL);
        g.al.assign(buf.begin() + 2 * sN + sL, buf.begin() + 2 * (sN + sL));
        g.depth.assign(buf.begin() + 2 * (sN + sL), buf.end());
    }
    return 0;
}

// output_saveResults (output.c:457-505) for the period ending at reportTime:
// interpolated point results, or with REPORT AVERAGES the period's averages
static void saveOutput(bool averages)
{
    double sys[6];
    G->router->stepTotals(G->sysStep);
    const bool multi = G->router->partition().active();
    if (multi) G->router->allreduceHost(G->sysStep, 6, 0);   // each rank's totals over what it owns
    // StepFlowTotals of this step: {flooding, outflow, dw, gw, ii, ex}
    sys[0] = G->sysStep[2];
    sys[1] = G->sysStep[3];
    sys[2] = G->sysStep[0];
    sys[3] = 0.0;
    sys[4] = 0.0;
    sys[5] = G->sysStep[1];
    Project& prj = *G->prj;
    double reportDate = prj.getDateTime(G->reportTime);
    if (reportDate < prj.opt.reportStart) return;     // (the averages keep accumulating)
    const float *nv = nullptr, *lv = nullptr, *an = nullptr, *al = nullptr;
    const double* depth = nullptr;
    if (averages) {
        if (G->router->avgTake(prj.ucfLength(), prj.ucfVolume(), prj.ucfFlow(), &an, &al, &nv, &lv, &depth)) {
            setErr(G->router->lastError(), G->router->lastErrorMsg());
            return;
        }
    } else {
        // interpolation weight between the bracketing steps (output.c:645)
        double f = (G->reportTime - G->oldRoutingTime) / (G->newRoutingTime - G->oldRoutingTime);
        if (G->router->packResults(f, prj.ucfLength(), prj.ucfVolume(), prj.ucfFlow(), &nv, &lv)) {
            setErr(G->router->lastError(), G->router->lastErrorMsg());
            return;
        }
    }
    GatheredResults g;
    if (multi) {
        if (syncError()) return;                    // every rank gathers, or none
        if (gatherResults(nv, lv, an, al, depth, g)) return;
        nv = g.nv.data();
        lv = g.lv.data();
        if (averages) {
            an = g.an.data();
            al = g.al.data();
            depth = g.depth.data();
        }
    }
    int e = G->out.saveResults(prj, reportDate, nv, lv, sys, an, al, depth, prj.ucfLength());
    if (e) setErr(e, "ERROR 309: cannot write to binary results file.");
    if (multi) syncError();                         // rank 0's write error stops every rank
}

static void updateAvg()      // output_updateAvgResults (output.c:857-907)
{
    Project& prj = *G->prj;
    if (G->router->avgUpdate(prj.ucfLength(), prj.ucfVolume(), prj.ucfFlow()))
        setErr(G->router->lastError(), G->router->lastErrorMsg());
}

static void saveResults()   // swmm5.c:579-613
{
    const bool averages = G->prj->rpt.averages != 0;
    if (G->newRoutingTime >= G->reportTime) {
        if (averages) {
            // the latest results join the period's averages when it ends
            // exactly now; past its end they open the next period's
            if (G->newRoutingTime == G->reportTime) updateAvg();
            if (!G->errorCode) saveOutput(true);
            if (!G->errorCode && G->newRoutingTime > G->reportTime) updateAvg();
        } else {
            saveOutput(false);
        }
        G->reportTime = G->reportTime + 1000 * (double)G->prj->opt.reportStep;
    } else if (averages) {
        updateAvg();
    }
}

int DLLEXPORT swmm_step(double* elapsedTime)
{
    if (elapsedTime) *elapsedTime = 0.0;
    if (!G) return 501;
    if (G->errorCode) return G->errorCode;
    if (!G->isOpen) return (G->errorCode = 501);
    if (!G->isStarted || G->hostOnly) return (G->errorCode = 502);
    if (G->stateSpent)
        return setErr(500, "ERROR 500: the state was advanced by swmmx_timeKernel (measurement only); "
                           "the run cannot continue.");
    if (G->newRoutingTime < G->routingDuration) {
        if (execRouting()) return G->errorCode;
    }
    if (G->saveFlag && (G->newRoutingTime >= G->reportTime || G->prj->rpt.averages)) saveResults();
    if (G->newRoutingTime < G->routingDuration) G->elapsedTime = G->newRoutingTime / kMsecPerDay;
    else G->elapsedTime = 0.0;
    if (elapsedTime) *elapsedTime = G->elapsedTime;
    return G->errorCode;
}

int DLLEXPORT swmmx_runSteps(int n, double* elapsedTime)
{
    double e = 0.0;
    for (int i = 0; i < n; i++) {
        int rc = swmm_step(&e);
        if (rc) return rc;
        if (e <= 0.0) break;
    }
    if (elapsedTime) *elapsedTime = e;
    return G ? G->errorCode : 501;
}

int DLLEXPORT swmm_stride(int strideStep, double* elapsedTime)   // swmm5.c:466-510
{
    if (elapsedTime) *elapsedTime = 0.0;
    if (!G) return 501;
    if (G->errorCode) return G->errorCode;
    if (!G->isOpen) return (G->errorCode = 501);
    if (!G->isStarted || G->hostOnly) return (G->errorCode = 502);
    if (G->stateSpent)
        return setErr(500, "ERROR 500: the state was advanced by swmmx_timeKernel (measurement only); "
                           "the run cannot continue.");
    Project& prj = *G->prj;
    double realRouteStep = prj.opt.routeStep;
    const double durPrev = G->routingDuration;           // in force at the last step's end
    double dur = G->newRoutingTime + 1000.0 * strideStep;
    if (prj.opt.totalDuration < dur) dur = prj.opt.totalDuration;
    G->routingDuration = dur;
    if (strideStep < prj.opt.routeStep) prj.opt.routeStep = strideStep;   // RouteStep = strideStep meanwhile
    if (G->router->repickStep(prj.opt.routeStep, durPrev, dur)) {
        prj.opt.routeStep = realRouteStep;               // leave the engine's step and duration as they were
        G->routingDuration = durPrev;
        return setErr(G->router->lastError(), G->router->lastErrorMsg());
    }
    double e = 0.0;
    do {
        swmm_step(&e);
    } while (e > 0.0 && !G->errorCode);
    prj.opt.routeStep = realRouteStep;
    G->routingDuration = prj.opt.totalDuration;
    if (!G->errorCode && G->router->repickStep(realRouteStep, dur, G->routingDuration))
        return setErr(G->router->lastError(), G->router->lastErrorMsg());
    if (G->newRoutingTime < prj.opt.totalDuration) G->elapsedTime = G->newRoutingTime / kMsecPerDay;
    else G->elapsedTime = 0.0;
    if (elapsedTime) *elapsedTime = G->elapsedTime;
    return G->errorCode;
}

static double computeFlowError()   // massbal.c:858-902
{
    Project& prj = *G->prj;
    double fs = 0.0;
    const Partition& part = G->router->partition();
    if (!part.active()) {
        for (int j = 0; j < prj.net.nNodes(); j++) fs += prj.st.newVolume[j];
        for (int j = 0; j < prj.net.nLinks(); j++) fs += prj.st.lNewVolume[j];
    } else {                         // each rank sums what it owns, then over the ranks
        for (int j = 0; j < prj.net.nNodes(); j++)
            if (part.nodeOwner[j] == part.rank) fs += prj.st.newVolume[j];
        for (int j = 0; j < prj.net.nLinks(); j++)
            if (part.linkOwner[j] == part.rank) fs += prj.st.lNewVolume[j];
        G->router->allreduceHost(&fs, 1, 0);
    }
    G->finalStorage = fs;
    double* T = G->flowTot;   // dw, ex, flooding, outflow, evap, seep
    double totalInflow = G->initStorage + 0.0 + 0.0;
    double totalOutflow = fs + T[2] + T[4] + T[5] + 0.0;
    if (T[0] >= 0.0) totalInflow += T[0]; else totalOutflow -= T[0];
    if (T[1] >= 0.0) totalInflow += T[1]; else totalOutflow -= T[1];
    if (T[3] >= 0.0) totalOutflow += T[3]; else totalInflow -= T[3];
    double pct = 0.0;
    if (fabs(totalInflow - totalOutflow) < 1.0) pct = kTiny;
    else if (fabs(totalInflow) > 0.0) pct = 100.0 * (1.0 - totalOutflow / totalInflow);
    else if (fabs(totalOutflow) > 0.0) pct = 100.0 * (totalInflow / totalOutflow - 1.0);
    return pct;
}

// Several GPUs: the hot start fields of the objects other ranks own into the
// host mirror (Router::download fills only this rank's), as gatherResults
// does: +inf in every slot this rank does not own, one min all-reduce
static int gatherMirror()
{
    const Partition& part = G->router->partition();
    Project& prj = *G->prj;
    State& st = prj.st;
    const size_t gN = prj.net.nNodes(), gL = prj.net.nLinks();
    const size_t P = prj.opt.ignoreQuality ? 0 : prj.net.nPollut();
    std::vector<double>* nodeArr[] = {&st.newDepth, &st.newLatFlow, &st.hrt};
    std::vector<double>* linkArr[] = {&st.lNewFlow, &st.lNewDepth, &st.setting};
    st.nNewQual.resize(P * gN);
    st.lNewQual.resize(P * gL);
    std::vector<double> buf;
    buf.reserve((3 + P) * (gN + gL));
    auto put = [&](const std::vector<double>& v, size_t n, bool nodes) {
        for (size_t k = 0; k < n; k++) {
            const size_t g = k % (nodes ? gN : gL);
            const int own = nodes ? part.nodeOwner[g] : part.linkOwner[g];
            buf.push_back(own == part.rank ? v[k] : INFINITY);
        }
    };
    for (auto* a : nodeArr) { a->resize(gN); put(*a, gN, true); }
    put(st.nNewQual, P * gN, true);
    for (auto* a : linkArr) { a->resize(gL); put(*a, gL, false); }
    put(st.lNewQual, P * gL, false);
    if (buf.size() > (size_t)0x7FFFFFFF) return setErr(500, "ERROR 500: hot start state too large to gather");
    if (G->router->allreduceHost(buf.data(), (int)buf.size(), 1))
        return setErr(G->router->lastError(), G->router->lastErrorMsg());
    size_t o = 0;
    auto take = [&](std::vector<double>& v, size_t n) {
        for (size_t k = 0; k < n; k++) v[k] = buf[o++];
    };
    for (auto* a : nodeArr) take(*a, gN);
    take(st.nNewQual, P * gN);
    for (auto* a : linkArr) take(*a, gL);
    take(st.lNewQual, P * gL);
    return 0;
}

static void writeReportSummary()   // massbal_report + stats_report (swmm5.c:628-632)
{
    if (!G->rpt || G->prj->rpt.disabled) return;
    Project& prj = *G->prj;
    long long iters = 0, nonConv = 0;
    int last = 0;
    G->router->counters(&iters, &nonConv, &last);
    if (G->router->partition().active()) {
        // statistics are per rank (owned objects); the tables need all of them
        fprintf(G->rpt, "\n  Summary tables are written by single-GPU runs only (rank %d of %d).\n",
                G->router->partition().rank, G->router->partition().nranks);
        return;
    }
    if (G->router->downloadStats(prj)) return;
    const double* T = G->flowTot;         // dw, ex, flooding, outflow, evap, seep
    ReportTotals t;
    t.dwInflow = T[0];
    t.exInflow = T[1];
    t.flooding = T[2];
    t.outflow = T[3];
    t.evapLoss = T[4];
    t.seepLoss = T[5];
    t.initStorage = G->initStorage;
    t.finalStorage = G->finalStorage;
    t.pctError = G->flowError;
    writeRunReport(G->rpt, prj, t, nonConv);
}

int DLLEXPORT swmm_end(void)   // swmm5.c:618-660
{
    if (!G || !G->isOpen) return 501;
    if (G->isStarted) {
        if (!G->hostOnly) {
            syncMirror();
            G->router->flowTotals(G->flowTot);
            G->router->allreduceHost(G->flowTot, 6, 0);   // per-rank totals (multi-GPU)
            G->flowError = computeFlowError();
            G->out.end(G->errorCode);                   // (output_end: its write errors are not reported)
            // after swmmx_timeKernel the state is not a routed one: no summary
            // tables and no hot start file from it (the report says why)
            if (G->stateSpent && G->rpt)
                fprintf(G->rpt, "\n  Summary tables and hot start file omitted: the state was advanced by "
                                "swmmx_timeKernel (measurement only).\n");
            if (!G->errorCode && !G->stateSpent) writeReportSummary();
            // hotstart_close (swmm5.c:647): the final state as a hot start
            // file (several GPUs: gathered from the owners, written by rank 0)
            const Partition& part = G->router->partition();
            if (part.active()) syncError();
            const bool saveHs = !G->errorCode && !G->stateSpent && !G->prj->hotstartSave.empty();
            if (saveHs && part.active()) gatherMirror();
            if (saveHs && !G->errorCode && (!part.active() || part.rank == 0) && G->prj->saveHotstart())
                setErr(G->prj->errorCode, G->prj->errorMsg);
            if (part.active()) syncError();
        }
        G->isStarted = false;
    }
    return G->errorCode;
}

int DLLEXPORT swmm_report(void) { return G ? G->errorCode : 501; }

int DLLEXPORT swmm_close(void)
{
    if (!G) return 0;
    G->out.close();
    if (G->rpt) fclose(G->rpt);
    G->rpt = nullptr;
    G->router.reset();
    delete G;
    G = nullptr;
    return 0;
}

int DLLEXPORT swmm_run(const char* f1, const char* f2, const char* f3)   // swmm5.c:186-252
{
    double elapsed = 0.0;
    swmm_open(f1, f2, f3);
    if (G && !G->errorCode) {
        swmm_start(1);
        if (!G->errorCode) {
            do {
                swmm_step(&elapsed);
            } while (elapsed > 0.0 && !G->errorCode);
        }
        swmm_end();
    }
    int err = G ? G->errorCode : 501;
    swmm_close();
    return err;
}

int DLLEXPORT swmm_getMassBalErr(float* runoffErr, float* flowErr, float* qualErr)
{
    if (runoffErr) *runoffErr = 0.0f;
    if (flowErr) *flowErr = 0.0f;
    if (qualErr) *qualErr = 0.0f;
    if (G && G->isOpen && !G->isStarted) {
        if (flowErr) *flowErr = (float)G->flowError;
        if (qualErr) *qualErr = (float)G->qualError;
    }
    return 0;
}

int DLLEXPORT swmm_getVersion(void) { return 52004; }

int DLLEXPORT swmm_getError(char* errMsg, int msgLen)
{
    if (!errMsg || msgLen <= 0) return G ? G->errorCode : 0;
    std::string m = G ? G->errorMsg : std::string();
    snprintf(errMsg, (size_t)msgLen, "%s", m.c_str());
    return G ? G->errorCode : 0;
}

int DLLEXPORT swmm_getWarnings(void) { return G ? G->prj->warnings : 0; }

int DLLEXPORT swmm_getCount(int objType)
{
    if (!G || !G->isOpen) return 0;
    switch (objType) {
    case swmm_GAGE: case swmm_SUBCATCH: return 0;
    case swmm_NODE: return G->prj->net.nNodes();
    case swmm_LINK: return G->prj->net.nLinks();
    default: return 0;
    }
}

void DLLEXPORT swmm_getName(int objType, int index, char* name, int size)
{
    if (!name || size <= 0) return;
    name[0] = '\0';
    if (!G || !G->isOpen) return;
    const Network& n = G->prj->net;
    if (objType == swmm_NODE && index >= 0 && index < n.nNodes()) snprintf(name, (size_t)size, "%s", n.nodeId[index].c_str());
    if (objType == swmm_LINK && index >= 0 && index < n.nLinks()) snprintf(name, (size_t)size, "%s", n.linkId[index].c_str());
}

int DLLEXPORT swmm_getIndex(int objType, const char* name)
{
    if (!G || !G->isOpen || !name) return -1;
    const Network& n = G->prj->net;
    if (objType == swmm_NODE) { auto it = n.nodeIndex.find(name); return it == n.nodeIndex.end() ? -1 : it->second; }
    if (objType == swmm_LINK) { auto it = n.linkIndex.find(name); return it == n.linkIndex.end() ? -1 : it->second; }
    return -1;
}

double DLLEXPORT swmm_getValue(int property, int index)   // swmm5.c:842-1213
{
    if (!G || !G->isOpen) return 0;
    Project& prj = *G->prj;
    if (property < 100) {
        switch (property) {
        case swmm_STARTDATE: return prj.opt.startDateTime;
        case swmm_CURRENTDATE: return prj.opt.startDateTime + G->elapsedTime;
        case swmm_ELAPSEDTIME: return G->elapsedTime;
        case swmm_ROUTESTEP: return prj.opt.routeStep;
        case swmm_MAXROUTESTEP: return prj.opt.routeStep;
        case swmm_REPORTSTEP: return prj.opt.reportStep;
        case swmm_TOTALSTEPS: return G->out.periods();
        case swmm_NOREPORT: return prj.rpt.disabled;
        case swmm_FLOWUNITS: return prj.opt.flowUnits;
        default: return 0;
        }
    }
    if (property >= 300 && property < 400) {
        if (index < 0 || index >= prj.net.nNodes()) return 0;
        const Network& n = prj.net;
        const State& s = prj.st;
        double uL = prj.ucfLength(), uQ = prj.ucfFlow();
        bool st = !s.newDepth.empty();
        if (property >= swmm_NODE_DEPTH && property <= swmm_NODE_OVERFLOW && G->isStarted &&
            !G->mirrorValid) {
            // one value straight from HBM instead of a full state download
            int f = -1;
            switch (property) {
            case swmm_NODE_DEPTH: case swmm_NODE_HEAD: f = Router::PK_NODE_DEPTH; break;
            case swmm_NODE_VOLUME: f = Router::PK_NODE_VOLUME; break;
            case swmm_NODE_LATFLOW: f = Router::PK_NODE_LATFLOW; break;
            case swmm_NODE_INFLOW: f = Router::PK_NODE_INFLOW; break;
            case swmm_NODE_OVERFLOW: f = Router::PK_NODE_OVERFLOW; break;
            }
            double v = 0.0;
            if (G->router->peek(f, index, &v)) return 0.0;
            switch (property) {
            case swmm_NODE_DEPTH: return v * uL;
            case swmm_NODE_HEAD: return (v + n.invertElev[index]) * uL;
            case swmm_NODE_VOLUME: return v * prj.ucfVolume();
            default: return v * uQ;
            }
        }
        switch (property) {
        case swmm_NODE_TYPE: return n.nodeType[index];
        case swmm_NODE_ELEV: return n.invertElev[index] * uL;
        case swmm_NODE_MAXDEPTH: return n.fullDepth[index] * uL;
        case swmm_NODE_DEPTH: return st ? s.newDepth[index] * uL : 0.0;
        case swmm_NODE_HEAD: return st ? (s.newDepth[index] + n.invertElev[index]) * uL : 0.0;
        case swmm_NODE_VOLUME: return st ? s.newVolume[index] * prj.ucfVolume() : 0.0;
        case swmm_NODE_LATFLOW: return st ? s.newLatFlow[index] * uQ : 0.0;
        case swmm_NODE_INFLOW: return st ? s.inflow[index] * uQ : 0.0;
        case swmm_NODE_OVERFLOW: return st ? s.overflow[index] * uQ : 0.0;
        case swmm_NODE_RPTFLAG: return n.rptFlag[index] > 0;
        default: return 0;
        }
    }
    if (property >= 400 && property < 500) {
        if (index < 0 || index >= prj.net.nLinks()) return 0;
        const Network& n = prj.net;
        const State& s = prj.st;
        double uL = prj.ucfLength(), uQ = prj.ucfFlow();
        bool st = !s.lNewDepth.empty();
        const Xsect& x = n.xsect[index];
        Geom g = geomOf(x, n.xTab.data());
        const double* ct = &SWX_CIRC_TABLES[0][0];
        bool dyn = (property >= swmm_LINK_FLOW && property <= swmm_LINK_TOPWIDTH) ||
                   property == swmm_LINK_SETTING;
        if (dyn && G->isStarted && !G->mirrorValid) {
            // flow / depth / setting of this link straight from HBM
            double q = 0.0, y = 0.0, set = 1.0;
            Router& r = *G->router;
            if (property == swmm_LINK_SETTING) {
                if (r.peek(Router::PK_LINK_SETTING, index, &set)) return 0.0;
                return set;
            }
            if (property != swmm_LINK_DEPTH && property != swmm_LINK_TOPWIDTH &&
                r.peek(Router::PK_LINK_FLOW, index, &q)) return 0.0;
            if (property != swmm_LINK_FLOW && r.peek(Router::PK_LINK_DEPTH, index, &y)) return 0.0;
            switch (property) {
            case swmm_LINK_FLOW: return q * uQ * (double)n.direction[index];
            case swmm_LINK_DEPTH: return y * uL;
            case swmm_LINK_TOPWIDTH: return getWofY(g, y, ct) * uL;
            case swmm_LINK_VELOCITY: {                     // link_getVelocity link.c:821-843
                double v = 0.0;
                if (y > 0.01 && n.linkType[index] == CONDUIT) {
                    double fl = fabs(q) / n.barrels[index];
                    double area = getAofY(g, y, ct);
                    if (area > kFudge) v = fl / area;
                }
                return v * uL;
            }
            default: return 0.0;
            }
        }
        switch (property) {
        case swmm_LINK_TYPE: return n.linkType[index];
        case swmm_LINK_NODE1: return n.node1[index];
        case swmm_LINK_NODE2: return n.node2[index];
        case swmm_LINK_LENGTH: return n.length[index] * uL;
        case swmm_LINK_SLOPE: return n.slope[index];
        case swmm_LINK_FULLDEPTH: return x.yFull * uL;
        case swmm_LINK_FULLFLOW: return n.qFull[index] * uQ;
        case swmm_LINK_FLOW: return st ? s.lNewFlow[index] * uQ * (double)n.direction[index] : 0.0;
        case swmm_LINK_VELOCITY: {
            if (!st || n.linkType[index] != CONDUIT) return 0.0;   // link_getVelocity: conduits only
            double depth = s.lNewDepth[index], v = 0.0;
            if (depth > 0.01) {
                double fl = fabs(s.lNewFlow[index]) / n.barrels[index];
                double area = getAofY(g, depth, ct);
                if (area > kFudge) v = fl / area;
            }
            return v * uL;
        }
        case swmm_LINK_DEPTH: return st ? s.lNewDepth[index] * uL : 0.0;
        case swmm_LINK_TOPWIDTH: return st ? getWofY(g, s.lNewDepth[index], ct) * uL : 0.0;
        case swmm_LINK_SETTING: return st ? s.setting[index] : 1.0;
        case swmm_LINK_RPTFLAG: return n.linkRpt[index] > 0;
        default: return 0;
        }
    }
    return 0;
}

void DLLEXPORT swmm_setValue(int property, int index, double value)
{
    if (!G || !G->isOpen) return;
    Project& prj = *G->prj;
    switch (property) {
    case swmm_NODE_LATFLOW:
        if (index < 0 || index >= prj.net.nNodes()) return;
        if (G->apiExtInflow.size() != (size_t)prj.net.nNodes()) G->apiExtInflow.assign(prj.net.nNodes(), 0.0);
        G->apiExtInflow[index] = value / prj.ucfFlow();
        G->constantInflow = false;
        return;
    case swmm_NODE_HEAD:                      // setOutfallStage (swmm5.c:1173-1188)
        if (index < 0 || index >= prj.net.nNodes() || prj.net.nodeType[index] != OUTFALL) return;
        prj.net.fixedStage[index] = value / prj.ucfLength();
        prj.net.outfallType[index] = O_FIXED;
        if (G->isStarted && G->router && G->router->setOutfallStage(index, prj.net.fixedStage[index]))
            setErr(G->router->lastError(), G->router->lastErrorMsg());
        return;
    case swmm_NODE_RPTFLAG:
        if (!G->isStarted && index >= 0 && index < prj.net.nNodes()) prj.net.rptFlag[index] = value > 0.0;
        return;
    case swmm_LINK_RPTFLAG:
        if (!G->isStarted && index >= 0 && index < prj.net.nLinks()) prj.net.linkRpt[index] = value > 0.0;
        return;
    case swmm_LINK_SETTING:
        return;   // conduit settings cannot be changed (swmm5.c:1323)
    case swmm_REPORTSTEP:
        if (!G->isStarted && value > 0) prj.opt.reportStep = (int)value;
        return;
    case swmm_NOREPORT:
        if (!G->isStarted) prj.rpt.disabled = value > 0.0;
        return;
    case swmm_ROUTESTEP:                      // setRoutingStep (swmm5.c:1360-1370)
        if (value <= 0.0) return;
        if (value <= prj.opt.minRouteStep) value = prj.opt.minRouteStep;
        prj.opt.courantFactor = 0.0;
        prj.opt.routeStep = value;
        if (G->isStarted && G->router && !G->hostOnly) {
            // the next step is fixed too: execRouting's clamp (swmm5.c:538-546)
            double dt = value;
            if (G->newRoutingTime + 1000.0 * dt > G->routingDuration) {
                dt = (G->routingDuration - G->newRoutingTime) / 1000.0;
                dt = (dt >= 1. / 1000.0) ? dt : 1. / 1000.0;
            }
            if (G->router->setRouteStep(value, dt)) setErr(G->router->lastError(), G->router->lastErrorMsg());
        }
        return;
    default:
        return;
    }
}

double DLLEXPORT swmm_getSavedValue(int property, int index, int period)   // swmm5.c:919-946
{
    if (!G || !G->isOpen || G->isStarted) return 0;
    if (period < 1 || period > G->out.periods()) return 0;
    if (property == swmm_CURRENTDATE) {
        double d = 0;
        G->out.readDate(period, &d);
        return d;
    }
    Network& n = G->prj->net;
    float v = 0.0f;
    if (property >= 300 && property < 400) {
        if (index < 0 || index >= n.nNodes() || !n.rptFlag[index]) return 0;
        int k = 0;
        for (int j = 0; j < index; j++) if (n.rptFlag[j]) k++;
        int var = -1;
        switch (property) {
        case swmm_NODE_DEPTH: var = 0; break;
        case swmm_NODE_HEAD: var = 1; break;
        case swmm_NODE_VOLUME: var = 2; break;
        case swmm_NODE_LATFLOW: var = 3; break;
        case swmm_NODE_INFLOW: var = 4; break;
        case swmm_NODE_OVERFLOW: var = 5; break;
        default: return 0;
        }
        G->out.readNodeVar(period, k, var, &v);
        return v;
    }
    if (property >= 400 && property < 500) {
        if (index < 0 || index >= n.nLinks() || !n.linkRpt[index]) return 0;
        int k = 0;
        for (int j = 0; j < index; j++) if (n.linkRpt[j]) k++;
        int var = -1;
        switch (property) {
        case swmm_LINK_FLOW: var = 0; break;
        case swmm_LINK_DEPTH: var = 1; break;
        case swmm_LINK_VELOCITY: var = 2; break;
        default: return 0;
        }
        G->out.readLinkVar(period, k, var, &v);
        return v;
    }
    return 0;
}

void DLLEXPORT swmm_writeLine(const char* line)
{
    if (G && G->isOpen && G->rpt && line) fprintf(G->rpt, "%s\n", line);
}

void DLLEXPORT swmm_decodeDate(double date, int* year, int* month, int* day, int* hour, int* minute,
                               int* second, int* dayOfWeek)
{
    decodeDate(date, year, month, day);
    decodeTime(date, hour, minute, second);
    *dayOfWeek = swx::dayOfWeek(date);
}

// ---------------------------------------------------------------- extensions
long DLLEXPORT swmmx_getArray(const char* name, double* dst, long n)
{
    if (!G || !G->isOpen || !name) return -1;
    if (G->isStarted && !G->hostOnly) syncMirror();
    Project& prj = *G->prj;
    State& s = prj.st;
    Network& net = prj.net;
    std::vector<double> tmp;
    const std::vector<double>* v = nullptr;
    std::string k(name);
#define ARR(nm, vec) if (k == nm) v = &vec;
    ARR("node.newDepth", s.newDepth) ARR("node.oldDepth", s.oldDepth) ARR("node.newVolume", s.newVolume)
    ARR("node.oldVolume", s.oldVolume) ARR("node.inflow", s.inflow) ARR("node.outflow", s.outflow)
    ARR("node.overflow", s.overflow) ARR("node.newLatFlow", s.newLatFlow) ARR("node.oldLatFlow", s.oldLatFlow)
    ARR("node.oldNetInflow", s.oldNetInflow) ARR("node.oldFlowInflow", s.oldFlowInflow)
    ARR("node.oldSurfArea", s.oldSurfArea) ARR("node.dYdT", s.dYdT)
    ARR("link.newFlow", s.lNewFlow) ARR("link.oldFlow", s.lOldFlow) ARR("link.newDepth", s.lNewDepth)
    ARR("link.oldDepth", s.lOldDepth) ARR("link.newVolume", s.lNewVolume) ARR("link.oldVolume", s.lOldVolume)
    ARR("link.surfArea1", s.surfArea1) ARR("link.surfArea2", s.surfArea2) ARR("link.froude", s.froude)
    ARR("link.dqdh", s.dqdh) ARR("link.a1", s.a1) ARR("link.a2", s.a2) ARR("link.q1", s.q1)
    ARR("link.q2", s.q1)   // under DW q2 == q1 (dwflow.c:285-286)
    ARR("link.setting", s.setting) ARR("link.evapLossRate", s.evapLossRate) ARR("link.seepLossRate", s.seepLossRate)
    ARR("node.newQual", s.nNewQual) ARR("node.oldQual", s.nOldQual) ARR("link.newQual", s.lNewQual)
    ARR("link.oldQual", s.lOldQual)
    ARR("node.invertElev", net.invertElev) ARR("node.fullDepth", net.fullDepth) ARR("node.surDepth", net.surDepth)
    ARR("node.pondedArea", net.pondedArea) ARR("node.crownElev", net.crownElev) ARR("node.fullVolume", net.fullVolume)
    ARR("node.fixedStage", net.fixedStage) ARR("node.initDepth", net.initDepth)
    ARR("link.offset1", net.offset1) ARR("link.offset2", net.offset2) ARR("link.q0", net.q0) ARR("link.qLimit", net.qLimit)
    ARR("link.cLossInlet", net.cLossInlet) ARR("link.cLossOutlet", net.cLossOutlet) ARR("link.cLossAvg", net.cLossAvg)
    ARR("link.seepRate", net.seepRate) ARR("link.length", net.length) ARR("link.roughness", net.roughness)
    ARR("link.modLength", net.modLength) ARR("link.roughFactor", net.roughFactor) ARR("link.slope", net.slope)
    ARR("link.beta", net.beta) ARR("link.qMax", net.qMax) ARR("link.qFull", net.qFull)
    if (k.compare(0, 5, "stat.") == 0) {          // run statistics (stats.c), device accumulators
        if (G->router && G->router->ok() && G->router->downloadStats(prj))
            return -1;
        RunStats& R = prj.stats;
        ARR("stat.node.avgDepth", R.avgDepth) ARR("stat.node.maxDepth", R.maxDepth)
        ARR("stat.node.maxDepthDate", R.maxDepthDate) ARR("stat.node.maxRptDepth", R.maxRptDepth)
        ARR("stat.node.volFlooded", R.volFlooded) ARR("stat.node.timeFlooded", R.timeFlooded)
        ARR("stat.node.timeSurcharged", R.timeSurcharged)
        ARR("stat.node.timeCourantCritical", R.timeCourantCritical) ARR("stat.node.totLatFlow", R.totLatFlow)
        ARR("stat.node.maxLatFlow", R.maxLatFlow) ARR("stat.node.maxInflow", R.maxInflow)
        ARR("stat.node.maxInflowDate", R.maxInflowDate) ARR("stat.node.maxOverflow", R.maxOverflow)
        ARR("stat.node.maxOverflowDate", R.maxOverflowDate) ARR("stat.node.maxPondedVol", R.maxPondedVol)
        ARR("stat.node.nonConvergedCount", R.nonConvergedCount)
        ARR("stat.node.inflowVolume", R.nodeInflowVol) ARR("stat.node.outflowVolume", R.nodeOutflowVol)
        ARR("stat.storage.initVol", R.stInitVol) ARR("stat.storage.avgVol", R.stAvgVol)
        ARR("stat.storage.maxVol", R.stMaxVol) ARR("stat.storage.maxFlow", R.stMaxFlow)
        ARR("stat.storage.evapLosses", R.stEvapLoss) ARR("stat.storage.exfilLosses", R.stExfilLoss)
        ARR("stat.storage.maxVolDate", R.stMaxVolDate)
        ARR("stat.pump.utilized", R.pUtilized) ARR("stat.pump.minFlow", R.pMinFlow)
        ARR("stat.pump.avgFlow", R.pAvgFlow) ARR("stat.pump.maxFlow", R.pMaxFlow)
        ARR("stat.pump.volume", R.pVolume) ARR("stat.pump.energy", R.pEnergy)
        ARR("stat.pump.offCurveLow", R.pOffLow) ARR("stat.pump.offCurveHigh", R.pOffHigh)
        ARR("stat.pump.startUps", R.pStartUps) ARR("stat.pump.totalPeriods", R.pPeriods)
        ARR("stat.outfall.avgFlow", R.outfallAvgFlow) ARR("stat.outfall.maxFlow", R.outfallMaxFlow)
        ARR("stat.outfall.totalPeriods", R.outfallPeriods) ARR("stat.outfall.totalLoad", R.outfallLoad)
        ARR("stat.link.maxFlow", R.lMaxFlow) ARR("stat.link.maxFlowDate", R.lMaxFlowDate)
        ARR("stat.link.maxVeloc", R.lMaxVeloc) ARR("stat.link.maxDepth", R.lMaxDepth)
        ARR("stat.link.timeNormalFlow", R.lTimeNormalFlow) ARR("stat.link.timeSurcharged", R.lTimeSurcharged)
        ARR("stat.link.timeInletControl", R.lTimeInletControl)
        ARR("stat.link.timeFullUpstream", R.lTimeFullUpstream)
        ARR("stat.link.timeFullDnstream", R.lTimeFullDnstream) ARR("stat.link.timeFullFlow", R.lTimeFullFlow)
        ARR("stat.link.timeCapacityLimited", R.lTimeCapacityLimited)
        ARR("stat.link.timeInFlowClass", R.lTimeInFlowClass)
        ARR("stat.link.timeCourantCritical", R.lTimeCourantCritical)
        ARR("stat.link.flowTurns", R.lFlowTurns) ARR("stat.link.flowTurnSign", R.lFlowTurnSign)
        if (k == "stat.sys") {
            tmp = {R.reportStepCount, R.routingTimeSpan, R.maxOutfallFlow, R.minTimeStep, R.maxTimeStep,
                   R.routingTime, R.steadyStateTime, R.timeStepCount, R.trialsCount};
            for (int j = 0; j < RunStats::kLevels; j++) tmp.push_back(R.timeStepCounts[j]);
            v = &tmp;
        }
    }
#undef ARR
    auto fromInt = [&](const std::vector<int>& iv) { tmp.assign(iv.begin(), iv.end()); v = &tmp; };
    if (k == "node.type") fromInt(net.nodeType);
    if (k == "node.degree") fromInt(net.degree);
    if (k == "node.outfallType") fromInt(net.outfallType);
    if (k == "node.outfallFlap") fromInt(net.outfallFlap);
    if (k == "link.type") fromInt(net.linkType);
    if (k == "link.node1") fromInt(net.node1);
    if (k == "link.node2") fromInt(net.node2);
    if (k == "link.hasFlapGate") fromInt(net.hasFlapGate);
    if (k == "link.direction") fromInt(net.direction);
    if (k == "link.barrels") fromInt(net.barrels);
    if (k == "link.hasLosses") fromInt(net.hasLosses);
    if (k == "link.superCritical") fromInt(net.superCritical);
    if (k == "link.flowClass") fromInt(s.flowClass);
    if (k == "link.fullState") fromInt(s.fullState);
    if (k == "link.normalFlow") fromInt(s.normalFlow);
    if (k == "link.capacityLimited") fromInt(s.capacityLimited);
    if (k == "node.converged") fromInt(s.converged);
    if (k.rfind("link.x", 0) == 0) {
        std::string f = k.substr(6);
        tmp.resize(net.nLinks());
        bool okf = true;
        for (int j = 0; j < net.nLinks(); j++) {
            const Xsect& x = net.xsect[j];
            if (f == "type") tmp[j] = x.type; else if (f == "yFull") tmp[j] = x.yFull;
            else if (f == "wMax") tmp[j] = x.wMax; else if (f == "ywMax") tmp[j] = x.ywMax;
            else if (f == "aFull") tmp[j] = x.aFull; else if (f == "rFull") tmp[j] = x.rFull;
            else if (f == "sFull") tmp[j] = x.sFull; else if (f == "sMax") tmp[j] = x.sMax;
            else if (f == "yBot") tmp[j] = x.yBot; else if (f == "aBot") tmp[j] = x.aBot;
            else if (f == "sBot") tmp[j] = x.sBot; else if (f == "rBot") tmp[j] = x.rBot;
            else if (f == "culvertCode") tmp[j] = x.culvertCode;
            else { okf = false; break; }
        }
        if (okf) v = &tmp;
    }
    if (k == "opt") {
        const Options& o = prj.opt;
        tmp = {o.routeStep, o.courantFactor, o.minRouteStep, o.minSurfArea, o.headTol, o.crownCutoff,
               o.lengtheningStep, o.evapRate, o.totalDuration, (double)o.reportStep, o.startDateTime,
               (double)o.maxTrials, (double)o.surchargeMethod, (double)o.inertDamping,
               (double)o.normalFlowLtd, (double)o.allowPonding};
        v = &tmp;
    }
    if (!v) return -1;
    long m = (long)v->size();
    if (dst) for (long i = 0; i < m && i < n; i++) dst[i] = (*v)[i];
    return m;
}

long DLLEXPORT swmmx_setArray(const char* name, const double* src, long n)
{
    if (!G || !G->isOpen || !name || !src) return -1;
    if (G->isStarted && !G->hostOnly) syncMirror();
    State& s = G->prj->st;
    std::vector<double>* v = nullptr;
    std::string k(name);
    if (k == "node.newDepth") v = &s.newDepth;
    if (k == "link.newFlow") v = &s.lNewFlow;
    if (k == "link.q1") v = &s.q1;
    if (!v) return -1;
    long m = std::min<long>((long)v->size(), n);
    for (long i = 0; i < m; i++) (*v)[i] = src[i];
    if (G->isStarted && !G->hostOnly) G->router->upload(*G->prj);
    return m;
}

int DLLEXPORT swmmx_exportState(const char* path)
{
    if (!G || !G->isOpen || !path) return 501;
    if (G->isStarted && !G->hostOnly) syncMirror();
    FILE* f = fopen(path, "wb");
    if (!f) return 303;
    fwrite("SWDUMP1\0", 1, 8, f);
    auto rec = [&](const std::string& name, char dt, const void* data, long long cnt) {
        char nm[48] = {0};
        snprintf(nm, sizeof nm, "%s", name.c_str());
        fwrite(nm, 1, 48, f);
        fwrite(&dt, 1, 1, f);
        fwrite(&cnt, 8, 1, f);
        fwrite(data, dt == 'd' ? 8 : 4, (size_t)cnt, f);
    };
    Project& prj = *G->prj;
    int counts[4] = {prj.net.nNodes(), prj.net.nLinks(), prj.net.nPollut(), 0};
    rec("counts", 'i', counts, 4);
    {   // the option records of oracle/refdump.c (same order)
        const Options& o = prj.opt;
        double od[12] = {o.routeStep, o.courantFactor, o.minRouteStep, o.minSurfArea, o.headTol,
                         o.crownCutoff, o.lengtheningStep, o.evapRate, o.totalDuration,
                         (double)o.reportStep, o.startDateTime, prj.st.variableStep};
        int oi[12] = {o.maxTrials, o.surchargeMethod, o.inertDamping, o.normalFlowLtd,
                      o.allowPonding, o.routeModel, o.forceMainEqn, o.flowUnits, o.unitSystem,
                      o.ignoreQuality, 0, 0};
        rec("opt.d", 'd', od, 12);
        rec("opt.i", 'i', oi, 12);
        int P = prj.net.nPollut();
        if (P > 0) {
            std::vector<double> kd(P), cd(P), ci(P);
            for (int p = 0; p < P; p++) {
                kd[p] = prj.net.pollut[p].kDecay;
                cd[p] = prj.net.pollut[p].cDWF;
                ci[p] = prj.net.pollut[p].cInit;
            }
            rec("pollut.kDecay", 'd', kd.data(), P);
            rec("pollut.dwfConcen", 'd', cd.data(), P);
            rec("pollut.initConcen", 'd', ci.data(), P);
        }
    }
    static const char* names[] = {
        "node.type", "node.degree", "node.outfallType", "node.outfallFlap", "node.invertElev",
        "node.initDepth", "node.fullDepth", "node.surDepth", "node.pondedArea", "node.crownElev",
        "node.fullVolume", "node.fixedStage", "node.newDepth", "node.oldDepth", "node.newVolume",
        "node.oldVolume", "node.inflow", "node.outflow", "node.newLatFlow", "node.oldLatFlow",
        "node.oldNetInflow", "node.oldFlowInflow", "node.overflow", "node.converged",
        "node.oldSurfArea", "node.dYdT",
        "link.type", "link.node1", "link.node2", "link.hasFlapGate", "link.direction", "link.flowClass",
        "link.xtype", "link.culvertCode", "link.barrels", "link.hasLosses", "link.superCritical",
        "link.offset1", "link.offset2", "link.q0", "link.qLimit", "link.cLossInlet", "link.cLossOutlet",
        "link.cLossAvg", "link.seepRate", "link.setting", "link.qFull", "link.yFull", "link.wMax",
        "link.ywMax", "link.aFull", "link.rFull", "link.sFull", "link.sMax", "link.yBot", "link.aBot",
        "link.sBot", "link.rBot", "link.length", "link.roughness", "link.modLength", "link.roughFactor",
        "link.slope", "link.beta", "link.qMax", "link.newFlow", "link.oldFlow", "link.newDepth",
        "link.oldDepth", "link.newVolume", "link.oldVolume", "link.a1", "link.a2", "link.q1", "link.q2",
        "link.froude", "link.dqdh", "link.surfArea1", "link.surfArea2", "link.fullState",
        "link.normalFlow", "link.capacityLimited", "node.newQual", "node.oldQual", "link.newQual",
        "link.oldQual", nullptr};
    std::vector<double> buf;
    for (int i = 0; names[i]; i++) {
        std::string nm = names[i];
        std::string q = nm;
        if (nm.rfind("link.", 0) == 0) {
            static const char* xf[] = {"yFull", "wMax", "ywMax", "aFull", "rFull", "sFull", "sMax",
                                       "yBot", "aBot", "sBot", "rBot", "culvertCode", nullptr};
            for (int k = 0; xf[k]; k++) if (nm == std::string("link.") + xf[k]) q = std::string("link.x") + xf[k];
            if (nm == "link.xtype") q = "link.xtype";
        }
        long m = swmmx_getArray(q.c_str(), nullptr, 0);
        if (m < 0) continue;
        buf.resize(std::max<long>(m, 1));
        swmmx_getArray(q.c_str(), buf.data(), m);
        bool isInt = nm == "node.type" || nm == "node.degree" || nm == "node.outfallType" ||
                     nm == "node.outfallFlap" || nm == "node.converged" || nm == "link.type" ||
                     nm == "link.node1" || nm == "link.node2" || nm == "link.hasFlapGate" ||
                     nm == "link.direction" || nm == "link.flowClass" || nm == "link.xtype" ||
                     nm == "link.culvertCode" || nm == "link.barrels" || nm == "link.hasLosses" ||
                     nm == "link.superCritical" || nm == "link.fullState" || nm == "link.normalFlow" ||
                     nm == "link.capacityLimited";
        if (isInt) {
            std::vector<int> iv(m);
            for (long j = 0; j < m; j++) iv[j] = (int)buf[j];
            rec(nm, 'i', iv.data(), m);
        } else {
            rec(nm == "opt" ? "opt.engine" : nm, 'd', buf.data(), m);
        }
    }
    fclose(f);
    return 0;
}

int DLLEXPORT swmmx_getCounters(long long* out, int n)
{
    if (!G || !out) return 0;
    long long v[19] = {G->totalStepCount, 0, 0, 0, G->prj->net.nLinks(), G->prj->net.nNodes(), 0, 0, 0, 0,
                       0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (G->router && G->router->ok()) {
        int last = 0;
        G->router->counters(&v[1], &v[2], &last);
        v[3] = last;
        double upd = 0, hot = 0, gat = 0, git = 0;
        G->router->timedWork(&upd, &hot, &gat, &git);
        v[6] = (long long)upd;
        v[7] = (long long)hot;
        v[8] = (long long)gat;
        v[9] = (long long)git;
        G->router->graphStats(&v[10]);
    }
    int m = n < 19 ? n : 19;
    for (int i = 0; i < m; i++) out[i] = v[i];
    return m;
}

long DLLEXPORT swmmx_evapReplay(const double* elapsedMsec, long n, double* rates)
{
    if (!G || !G->isStarted || !G->hostOnly || !elapsedMsec || !rates || n < 0) return -502;
    Project& prj = *G->prj;
    for (long i = 0; i < n; i++) {
        const double r = prj.climateSetState(prj.getDateTime(elapsedMsec[i]));
        if (prj.errorCode) return -(long)prj.errorCode;
        rates[i] = r;
    }
    return n;
}

int DLLEXPORT swmmx_setTiming(int mode)
{
    if (!G || !G->router) return 502;
    G->router->setTiming(mode != 0);
    return 0;
}

int DLLEXPORT swmmx_getKernelTimes(double* out, int n)
{
    if (!G || !G->router) return 0;
    return G->router->kernelTimes(out, n);
}

int DLLEXPORT swmmx_getIterationStats(double* out, int n)
{
    if (!G || !G->router) return 0;
    return G->router->iterationStats(out, n);
}

int DLLEXPORT swmmx_getKernelBytes(double* out, int n)
{
    if (!G || !G->router) return 0;
    return G->router->kernelBytes(out, n);
}

int DLLEXPORT swmmx_xsect(int type, const double* p, double ucf, int fn, const double* x, double* y,
                          int n, int device)
{
    Xsect xs;
    double q[4] = {p[0], p[1], p[2], p[3]};
    if (type < 0 || type > X_STREET || !setXsectParams(xs, type, q, ucf)) return 211;
    if (fn == 0) {
        const double v[11] = {xs.yFull, xs.wMax, xs.ywMax, xs.aFull, xs.rFull, xs.sFull, xs.sMax,
                              xs.yBot, xs.aBot, xs.sBot, xs.rBot};
        for (int i = 0; i < 11 && i < n; i++) y[i] = v[i];
        return 0;
    }
    Geom g = geomOf(xs);
    if (device) return xsectEvalDevice(g, fn, x, y, n);
    for (int i = 0; i < n; i++) y[i] = evalXsect(g, fn, x[i], &SWX_CIRC_TABLES[0][0]);
    return 0;
}

int DLLEXPORT swmmx_getBackend(char* buf, int size)
{
    std::string s = (G && G->router && G->router->ok()) ? G->router->deviceName() : std::string("none");
    if (buf && size > 0) snprintf(buf, (size_t)size, "%s", s.c_str());
    return 0;
}

int DLLEXPORT swmmx_timeKernel(int which, int reps, double* avgUs)
{
    if (!G || !G->router || !G->router->ok() || !avgUs) return 502;
    G->mirrorValid = false;
    // the replays advance the live state (the first passes rotate it; storage
    // exfiltration moves its Green-Ampt state): no routing step may follow
    G->stateSpent = true;
    return G->router->timeKernel(which, reps, avgUs);
}

int DLLEXPORT swmmx_ncclUniqueId(void* out, int bytes)
{
    if (!out || bytes < (int)sizeof(ncclUniqueId)) return -1;
    ncclUniqueId id;
    // the root's bootstrap address: the loopback interface unless the caller
    // chose one (single node; an unset interface makes RCCL probe the host's)
    setenv("NCCL_SOCKET_IFNAME", "lo", 0);
    if (ncclGetUniqueId(&id) != ncclSuccess) return -2;
    memcpy(out, &id, sizeof id);
    return (int)sizeof id;
}

int DLLEXPORT swmmx_setPartition(int rank, int nranks, const void* ncclId, int idBytes)
{
    if (nranks < 1 || rank < 0 || rank >= nranks) return 500;
    gPart = Partition();
    gPart.rank = rank;
    gPart.nranks = nranks;
    gPart.transport = XCHG_RCCL;
    if (ncclId && idBytes > 0) {
        const unsigned char* b = (const unsigned char*)ncclId;
        gPart.ncclId.assign(b, b + idBytes);
        gPart.forced = (nranks == 1);     // one rank through the RCCL path: tests
    }
    return 0;
}

int DLLEXPORT swmmx_setExchange(int (*fn)(double*, long, int, void*), void* user)
{
    gPart.transport = fn ? XCHG_HOST : XCHG_RCCL;
    gPart.xchg = fn;
    gPart.xuser = user;
    return 0;
}

int DLLEXPORT swmmx_setPartitionWeights(const double* w, int n)
{
    if (n < 0 || (n > 0 && !w)) return 500;
    gPart.weight.assign(w, w + n);
    return 0;
}

int DLLEXPORT swmmx_setPartitionMode(int mode)
{
    if (mode != PART_CONTIGUOUS && mode != PART_TWO_REGION) return 500;
    gPart.mode = mode;
    return 0;
}

int DLLEXPORT swmmx_getNodeWork(double* out, int n)
{
    if (!G || !G->router || !G->router->ok() || !out) return -1;
    for (int i = 0; i < n; i++) out[i] = 0.0;
    if (G->router->nodeWork(out, n)) return -1;
    return G->prj->net.nNodes();
}

int DLLEXPORT swmmx_getConduitWork(double* out, int n)
{
    if (!G || !G->router || !G->router->ok() || !out) return -1;
    for (int i = 0; i < n; i++) out[i] = 0.0;
    if (G->router->nodeWork(out, n, true)) return -1;
    return G->prj->net.nNodes();
}

int DLLEXPORT swmmx_setTransport(int kind)
{
    if (kind < XCHG_RCCL || kind > XCHG_IPC) return 500;
    if (kind == XCHG_HOST && !gPart.xchg) return 500;
    gPart.transport = kind;
    return 0;
}

int DLLEXPORT swmmx_getTransport(char* buf, int size)
{
    std::string s = (G && G->router && G->router->ok()) ? G->router->transport() : std::string("none");
    if (buf && size > 0) snprintf(buf, (size_t)size, "%s", s.c_str());
    return 0;
}

int DLLEXPORT swmmx_getOwner(int objType, int* out, int n)
{
    if (!G || !G->prj) return -1;
    Partition p;
    p.rank = gPart.rank;
    p.nranks = gPart.nranks;
    p.weight = gPart.weight;
    p.mode = gPart.mode;
    std::string m;
    if (buildPartition(G->prj->net, p, &m)) return -1;
    const std::vector<int>& v = (objType == swmm_NODE) ? p.nodeOwner : p.linkOwner;
    int k = std::min(n, (int)v.size());
    for (int i = 0; i < k; i++) out[i] = v[i];
    return (int)v.size();
}

long DLLEXPORT swmmx_getPartition(const char* name, int* out, long n)
{
    if (!G || !G->prj || !name) return -1;
    Partition p;
    p.rank = gPart.rank;
    p.nranks = gPart.nranks;
    p.weight = gPart.weight;
    p.mode = gPart.mode;
    std::string m;
    if (buildPartition(G->prj->net, p, &m)) return -1;
    std::vector<int> rowptr, csr, hg;
    const std::string nm = name;
    const std::vector<int>* v = nullptr;
    if (nm == "lnode") v = &p.lnode;
    else if (nm == "llink") v = &p.llink;
    else if (nm == "lghost") v = &p.lghost;
    else if (nm == "nbr") v = &p.nbr;
    else if (nm == "sendOff") v = &p.sendOff;
    else if (nm == "sendLink") v = &p.sendLink;
    else if (nm == "recvOff") v = &p.recvOff;
    else if (nm == "hasGhost") { hg.assign(p.hasGhost.begin(), p.hasGhost.end()); v = &hg; }
    else if (nm == "rowptr" || nm == "csr") {
        buildLocalCsr(G->prj->net, p, true, rowptr, csr);
        v = (nm == "rowptr") ? &rowptr : &csr;
    } else return -1;
    long k = std::min<long>(n, (long)v->size());
    for (long i = 0; i < k && out; i++) out[i] = (*v)[i];
    return (long)v->size();
}

int DLLEXPORT swmmx_setDevice(int ordinal)
{
    gDevice = ordinal;
    return 0;
}

}  // extern "C"
