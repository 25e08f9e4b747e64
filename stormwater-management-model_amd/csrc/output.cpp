// output.cpp -- binary results writer/reader, byte-compatible with the
// reference's .out format (src/solver/output.c; the layout is what the
// reference's own reader library src/outfile/swmm_output.c expects).
#include "output.h"

#include <cmath>
#include <cstring>

#include "xsect.h"

namespace swx {

static const int kMagic = 516114522;   // consts.h:20
static const int kVersion = 52004;     // consts.h:19
static const int kMaxSysResults = 15;  // enums.h:224

OutFile::~OutFile() { close(); }

static void w4(FILE* f, int k) { fwrite(&k, 4, 1, f); }
static void wf(FILE* f, float x) { fwrite(&x, 4, 1, f); }
static void wid(FILE* f, const std::string& s)
{
    w4(f, (int)s.size());
    fwrite(s.data(), 1, s.size(), f);
}

int OutFile::open(const std::string& path, Project& prj)  // output.c:121-405
{
    Network& net = prj.net;
    path_ = path;
    f_ = fopen(path.c_str(), "w+b");
    if (!f_) return 307;
    nPoll_ = prj.opt.ignoreQuality ? 0 : net.nPollut();
    nNodeVars_ = 6 + nPoll_;
    nLinkVars_ = 5 + nPoll_;
    int nSubVars = 8 + nPoll_;
    nNodes_ = nLinks_ = 0;
    for (int j = 0; j < net.nNodes(); j++) if (net.rptFlag[j]) nNodes_++;
    for (int j = 0; j < net.nLinks(); j++) if (net.linkRpt[j]) nLinks_++;
    long long numResults = (long long)nNodes_ * nNodeVars_ + (long long)nLinks_ * nLinkVars_ + kMaxSysResults;
    bytesPerPeriod_ = 8 + numResults * 4;
    nPeriods_ = 0;
    double uL = prj.ucfLength();

    w4(f_, kMagic);
    w4(f_, kVersion);
    w4(f_, prj.opt.flowUnits);
    w4(f_, 0);          // subcatchments
    w4(f_, nNodes_);
    w4(f_, nLinks_);
    w4(f_, nPoll_);
    idStart_ = (int)ftell(f_);
    for (int j = 0; j < net.nNodes(); j++) if (net.rptFlag[j]) wid(f_, net.nodeId[j]);
    for (int j = 0; j < net.nLinks(); j++) if (net.linkRpt[j]) wid(f_, net.linkId[j]);
    for (int p = 0; p < nPoll_; p++) wid(f_, net.pollut[p].id);
    for (int p = 0; p < nPoll_; p++) w4(f_, net.pollut[p].units);
    inputStart_ = (int)ftell(f_);
    w4(f_, 1);          // subcatchment area block (no subcatchments)
    w4(f_, 1);          // INPUT_AREA
    w4(f_, 3); w4(f_, 0); w4(f_, 2); w4(f_, 3);     // node: type, invert, max depth
    for (int j = 0; j < net.nNodes(); j++) {
        if (!net.rptFlag[j]) continue;
        w4(f_, net.nodeType[j]);
        wf(f_, (float)(net.invertElev[j] * uL));
        wf(f_, (float)(net.fullDepth[j] * uL));
    }
    w4(f_, 5); w4(f_, 0); w4(f_, 4); w4(f_, 4); w4(f_, 3); w4(f_, 5);   // link input codes
    for (int j = 0; j < net.nLinks(); j++) {
        if (!net.linkRpt[j]) continue;
        float r[4] = {0.0f, 0.0f, 0.0f, 0.0f};        // pumps: all zero (output.c:281-284)
        int k = net.linkType[j];
        if (k != PUMP) {
            r[0] = (float)(net.offset1[j] * uL);
            r[1] = (float)(net.offset2[j] * uL);
            if (net.direction[j] < 0) std::swap(r[0], r[1]);
            r[2] = (k == OUTLET) ? 0.0f : (float)(net.xsect[j].yFull * uL);
            r[3] = (k == CONDUIT) ? (float)(net.length[j] * uL) : 0.0f;
        }
        w4(f_, net.linkType[j]);
        fwrite(r, 4, 4, f_);
    }
    w4(f_, nSubVars);
    for (int k = 0; k < 8; k++) w4(f_, k);
    for (int p = 0; p < nPoll_; p++) w4(f_, 8 + p);
    w4(f_, nNodeVars_);
    for (int k = 0; k < 6; k++) w4(f_, k);
    for (int p = 0; p < nPoll_; p++) w4(f_, 6 + p);
    w4(f_, nLinkVars_);
    for (int k = 0; k < 5; k++) w4(f_, k);
    for (int p = 0; p < nPoll_; p++) w4(f_, 5 + p);
    w4(f_, kMaxSysResults);
    for (int k = 0; k < kMaxSysResults; k++) w4(f_, k);
    double z = (double)prj.opt.reportStep / 86400.0;
    if (prj.opt.startDateTime + z > prj.opt.reportStart) z = prj.opt.startDateTime;
    else {
        z = floor((prj.opt.reportStart - prj.opt.startDateTime) / z) - 1.0;
        z = prj.opt.startDateTime + z * (double)prj.opt.reportStep / 86400.0;
    }
    fwrite(&z, 8, 1, f_);
    w4(f_, prj.opt.reportStep);
    outputStart_ = (int)ftell(f_);
    return ferror(f_) ? 309 : 0;
}

int OutFile::saveResults(Project& prj, double reportDate, const float* nodeVals, const float* linkVals,
                         const double sys[6], const float* avgNode, const float* avgLink, const double* depth,
                         double uL)   // output.c:457-505, 636-695 (averages: 911-955)
{
    if (!f_) return 0;
    Network& net = prj.net;
    int nn = net.nNodes(), nl = net.nLinks(), P = nPoll_;
    const int nv = 6 + P, lv = 5 + P;
    double uQ = prj.ucfFlow();
    float sysr[kMaxSysResults];
    for (float& x : sysr) x = 0.0f;
    fwrite(&reportDate, 8, 1, f_);
    std::vector<double>& rpt = prj.stats.maxRptDepth;
    if ((int)rpt.size() != nn) rpt.assign(nn, 0.0);
    // node rows (node_getResults node.c:497-528, packed on the device)
    if (avgNode) {
        // averaged rows of the reported objects; the maximum reported depth
        // takes each node's current depth and the system storage its current
        // volume (output.c:914-950)
        for (int j = 0; j < nn; j++)
            if (net.rptFlag[j]) fwrite(avgNode + (size_t)j * nv, 4, nNodeVars_, f_);
        for (int j = 0; j < nn; j++) {
            const double y = depth[j] * uL;
            rpt[j] = (rpt[j] >= y) ? rpt[j] : y;
            sysr[12] += nodeVals[(size_t)j * nv + 2];
        }
        for (int j = 0; j < nl; j++)
            if (net.linkRpt[j]) fwrite(avgLink + (size_t)j * lv, 4, nLinkVars_, f_);
        for (int j = 0; j < nl; j++) sysr[12] += linkVals[(size_t)j * lv + 3];
    } else {
        for (int j = 0; j < nn; j++) {
            const float* x = nodeVals + (size_t)j * nv;
            if (net.rptFlag[j]) fwrite(x, 4, nNodeVars_, f_);
            // stats_updateMaxNodeDepth (stats.c:436-445) with the reported value
            rpt[j] = (rpt[j] >= (double)x[0]) ? rpt[j] : (double)x[0];
            sysr[12] += x[2];
        }
        // link rows (link_getResults link.c:674-724); system storage adds every
        // link's volume in link order (output.c:668-671)
        for (int j = 0; j < nl; j++) {
            const float* x = linkVals + (size_t)j * lv;
            if (net.linkRpt[j]) fwrite(x, 4, nLinkVars_, f_);
            sysr[12] += x[3];
        }
    }
    sysr[10] = (float)(sys[0] * uQ);
    sysr[11] = (float)(sys[1] * uQ);
    sysr[5] = (float)(sys[2] * uQ);
    sysr[6] = (float)(sys[3] * uQ);
    sysr[7] = (float)(sys[4] * uQ);
    sysr[8] = (float)(sys[5] * uQ);
    sysr[9] = sysr[4] + sysr[5] + sysr[6] + sysr[7] + sysr[8];
    fwrite(sysr, 4, kMaxSysResults, f_);
    nPeriods_++;
    return ferror(f_) ? 309 : 0;
}

int OutFile::end(int errorCode)   // output.c:515-535
{
    if (!f_) return 0;
    w4(f_, idStart_);
    w4(f_, inputStart_);
    w4(f_, outputStart_);
    w4(f_, nPeriods_);
    w4(f_, errorCode);
    w4(f_, kMagic);
    fflush(f_);
    return ferror(f_) ? 309 : 0;
}

void OutFile::close()
{
    if (f_) fclose(f_);
    f_ = nullptr;
}

bool OutFile::readDate(int period, double* date)
{
    if (!f_ || period < 1 || period > nPeriods_) return false;
    long long pos = outputStart_ + (long long)(period - 1) * bytesPerPeriod_;
    fseek(f_, (long)pos, SEEK_SET);
    return fread(date, 8, 1, f_) == 1;
}

bool OutFile::readNodeVar(int period, int idx, int var, float* v)
{
    if (!f_ || period < 1 || period > nPeriods_ || idx < 0 || idx >= nNodes_) return false;
    long long pos = outputStart_ + (long long)(period - 1) * bytesPerPeriod_ + 8 +
                    ((long long)idx * nNodeVars_ + var) * 4;
    fseek(f_, (long)pos, SEEK_SET);
    return fread(v, 4, 1, f_) == 1;
}

bool OutFile::readLinkVar(int period, int idx, int var, float* v)
{
    if (!f_ || period < 1 || period > nPeriods_ || idx < 0 || idx >= nLinks_) return false;
    long long pos = outputStart_ + (long long)(period - 1) * bytesPerPeriod_ + 8 +
                    ((long long)nNodes_ * nNodeVars_ + (long long)idx * nLinkVars_ + var) * 4;
    fseek(f_, (long)pos, SEEK_SET);
    return fread(v, 4, 1, f_) == 1;
}

}  // namespace swx
