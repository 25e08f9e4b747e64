// report.h -- end-of-run report tables (the reference's massbal_report +
// stats_report, written by swmm_end; src/solver/report.c, statsrpt.c).
//
// Layout and number formats reproduce the reference's report file so that
// tools parsing it keep working; values come from the device run statistics
// (prj.stats, Router::downloadStats) and the flow totals.
#pragma once

#include <cstdio>

#include "project.h"

namespace swx {

struct ReportTotals {            // TRoutingTotals (objects.h) in ft3
    double dwInflow = 0, wwInflow = 0, gwInflow = 0, iiInflow = 0, exInflow = 0;
    double flooding = 0, outflow = 0, evapLoss = 0, seepLoss = 0;
    double initStorage = 0, finalStorage = 0, pctError = 0;
};

// Writes the continuity, accuracy-statistics and summary tables.  Expects
// prj.stats to be current; adds the final node volumes to the node outflow
// totals (massbal_getStorage(TRUE), massbal.c:649-653) on the way.
void writeRunReport(FILE* f, Project& prj, const ReportTotals& tot, long long nonConvergeCount);

}  // namespace swx
