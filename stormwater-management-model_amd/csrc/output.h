// output.h -- binary results file (.out) in the reference's exact layout
// (src/solver/output.c:121-535: header, IDs, input summary, per-period
// float32 node/link/system results, closing records).
#pragma once

#include <cstdio>
#include <string>
#include <vector>

#include "project.h"

namespace swx {

class OutFile {
public:
    ~OutFile();
    int open(const std::string& path, Project& prj);
    // write one reporting period from the device-packed rows (Router::
    // packResults: nodes 6 + P floats, links 5 + P floats, all objects);
    // sysFlows = {flooding, outflow, dwInflow, gwInflow, iiInflow, exInflow}
    // rates of the bracketing step (StepFlowTotals)
    // REPORT AVERAGES (output_saveAvgResults, output.c:911-955): the rows come
    // from avgNode / avgLink, while nodeVals / linkVals hold the current state
    // (f = 1) for the system storage and depth (ft, times uL) the reported
    // maximum depth
    int saveResults(Project& prj, double reportDate, const float* nodeVals, const float* linkVals,
                    const double sysFlows[6], const float* avgNode = nullptr, const float* avgLink = nullptr,
                    const double* depth = nullptr, double uL = 1.0);
    int end(int errorCode);
    void close();
    int periods() const { return nPeriods_; }
    // random access to saved periods (swmm_getSavedValue, swmm5.c:919-946)
    bool readDate(int period, double* date);
    bool readNodeVar(int period, int nodeOutIdx, int var, float* v);
    bool readLinkVar(int period, int linkOutIdx, int var, float* v);
    int nodeVars() const { return nNodeVars_; }
    int linkVars() const { return nLinkVars_; }

private:
    FILE* f_ = nullptr;
    std::string path_;
    int idStart_ = 0, inputStart_ = 0, outputStart_ = 0;
    int nPeriods_ = 0, nNodes_ = 0, nLinks_ = 0, nPoll_ = 0;
    int nNodeVars_ = 0, nLinkVars_ = 0;
    long long bytesPerPeriod_ = 0;
    std::vector<float> buf_;
};

}  // namespace swx
