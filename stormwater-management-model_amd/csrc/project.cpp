// project.cpp -- .inp reader, validation and initial state (host only).
//
// Restates the parts of the reference's input/project/link/node/xsect/
// flowrout modules that define every constant and initial value the routing
// kernels read.  The reader is our own two-pass,
// hash-map based design (O(N) -- the reference's fixed 1999-bucket ID hash
// makes swmm_open O(N^2): 157 s at 1M conduits); the derived values follow
// the reference arithmetic exactly so that tests/test_host_init.py can assert
// bit-equality of every parameter and initial state value.
//
// Supported input: [TITLE] [OPTIONS] [EVAPORATION] (CONSTANT) [JUNCTIONS]
// [OUTFALLS] (FREE/NORMAL/FIXED/TIMESERIES) [CONDUITS] [XSECTIONS]
// (CIRCULAR, FORCE_MAIN excluded, RECT_CLOSED, RECT_OPEN, TRAPEZOIDAL,
// TRIANGULAR) [LOSSES] [POLLUTANTS] [INFLOWS] [DWF] [PATTERNS] [TIMESERIES]
// [REPORT]; map/graphics sections are skipped.  Anything else fails loudly
// with ERR_INPUT naming the section (never silently ignored).
#include "project.h"
#include "storage.h"
#include "regulators.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <algorithm>

#include "xsect.h"

namespace swx {

// ===================================================================== dates
static const int kDateDelta = 693594;          // datetime.c:40
static const double kSecsPerDay = 86400.;      // datetime.c:41
static const int kDaysPerMonth[2][12] = {{31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31},
                                         {31, 29, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31}};
static int isLeap(int y) { return ((y % 4 == 0) && ((y % 100 != 0) || (y % 400 == 0))) ? 1 : 0; }

double encodeDate(int year, int month, int day)  // datetime.c:108-132
{
    int i = isLeap(year);
    if (year >= 1 && year <= 9999 && month >= 1 && month <= 12 && day >= 1 &&
        day <= kDaysPerMonth[i][month - 1]) {
        for (int j = 0; j < month - 1; j++) day += kDaysPerMonth[i][j];
        i = year - 1;
        i = i * 365 + i / 4 - i / 100 + i / 400 + day - kDateDelta;
        return i;
    }
    return -kDateDelta;
}

double encodeTime(int hour, int minute, int second)  // datetime.c:136-152
{
    if (hour >= 0 && minute >= 0 && second >= 0) {
        int s = hour * 3600 + minute * 60 + second;
        return (double)s / kSecsPerDay;
    }
    return 0.0;
}

static int findMonth(const char* m)
{
    static const char* names[] = {"JAN", "FEB", "MAR", "APR", "MAY", "JUN",
                                  "JUL", "AUG", "SEP", "OCT", "NOV", "DEC"};
    for (int i = 0; i < 12; i++)
        if (strncasecmp(m, names[i], 3) == 0) return i + 1;
    return -1;
}

bool strToDate(const char* s, double* d)  // datetime.c:284-334 (M/D/Y format)
{
    int yr = 0, mon = 0, day = 0;
    char month[4] = {0};
    char sep1, sep2;
    *d = -kDateDelta;
    if (strchr(s, '-') || strchr(s, '/')) {
        int n = sscanf(s, "%d%c%d%c%d", &mon, &sep1, &day, &sep2, &yr);
        if (n < 3) {
            mon = 0;
            n = sscanf(s, "%3s%c%d%c%d", month, &sep1, &day, &sep2, &yr);
            if (n < 3) return false;
        }
        if (mon == 0) mon = findMonth(month);
        *d = encodeDate(yr, mon, day);
    }
    return *d != -kDateDelta;
}

bool strToTime(const char* s, double* t)  // datetime.c:338-365
{
    char* endptr;
    *t = strtod(s, &endptr);
    if (*endptr == 0) {
        *t /= 24.0;
        return true;
    }
    int hr = 0, min = 0, sec = 0;
    *t = 0.0;
    int n = sscanf(s, "%d:%d:%d", &hr, &min, &sec);
    if (n == 0) return false;
    *t = encodeTime(hr, min, sec);
    return hr >= 0 && min >= 0 && sec >= 0;
}

static void divMod(int n, int d, int* result, int* remainder)
{
    if (d == 0) { *result = 0; *remainder = 0; }
    else { *result = n / d; *remainder = n - d * (*result); }
}

void decodeDate(double date, int* year, int* month, int* day)  // datetime.c:158-220
{
    const int D1 = 365, D4 = D1 * 4 + 1, D100 = D4 * 25 - 1, D400 = D100 * 4 + 1;
    int t = (int)(floor(date)) + kDateDelta, y, m, d, i, k;
    if (t <= 0) { *year = 0; *month = 1; *day = 1; return; }
    t--;
    y = 1;
    while (t >= D400) { t -= D400; y += 400; }
    divMod(t, D100, &i, &d);
    if (i == 4) { i--; d += D100; }
    y += i * 100;
    divMod(d, D4, &i, &d);
    y += i * 4;
    divMod(d, D1, &i, &d);
    if (i == 4) { i--; d += D1; }
    y += i;
    k = isLeap(y);
    m = 1;
    for (;;) {
        i = kDaysPerMonth[k][m - 1];
        if (d < i) break;
        d -= i;
        m++;
    }
    *year = y; *month = m; *day = d + 1;
}

void decodeTime(double time, int* h, int* m, int* s)  // datetime.c:224-241
{
    double fracDay = (time - floor(time)) * kSecsPerDay;
    int secs = (int)(floor(fracDay + 0.5)), mins;
    if (secs >= 86400) secs = 86399;
    divMod(secs, 60, &mins, s);
    divMod(mins, 60, h, m);
    if (*h > 23) *h = 0;
}

double addSeconds(double date1, double seconds)  // datetime.c:381-393
{
    double d = floor(date1);
    int h, m, s;
    decodeTime(date1, &h, &m, &s);
    return d + (3600.0 * h + 60.0 * m + s + seconds) / kSecsPerDay;
}

int monthOfYear(double date) { int y, m, d; decodeDate(date, &y, &m, &d); return m; }
int dayOfWeek(double date) { int t = (int)(floor(date)) + kDateDelta; return (t % 7) + 1; }
int hourOfDay(double date) { int h, m, s; decodeTime(date, &h, &m, &s); return h; }

// ============================================================== tokenising
// input.c:getTokens semantics: ';' starts a comment, whitespace separates,
// a double quote starts a token that runs to the next quote.
static int tokenize(char* s, std::vector<char*>& tok)
{
    tok.clear();
    char* c = strchr(s, ';');
    if (c) *c = '\0';
    int len = (int)strlen(s);
    const char* sep = " \t\n\r";
    while (len > 0) {
        int m = (int)strcspn(s, sep);
        if (m == 0) {
            s++;
        } else {
            if (*s == '"') {
                s++;
                len--;
                m = (int)strcspn(s, "\"\n");
            }
            s[m] = '\0';
            tok.push_back(s);
            s += m + 1;
        }
        len -= m + 1;
    }
    return (int)tok.size();
}

// input.c:match -- keyword is a case-insensitive prefix of str
static bool kmatch(const char* str, const char* kw)
{
    if (!kw[0]) return false;
    while (*str == ' ') str++;
    for (; *kw; kw++, str++)
        if (!*str || toupper((unsigned char)*str) != toupper((unsigned char)*kw)) return false;
    return true;
}
static int kfind(const char* s, const char* const* kws)
{
    for (int i = 0; kws[i]; i++)
        if (kmatch(s, kws[i])) return i;
    return -1;
}
static bool getDouble(const char* s, double* y)
{
    char* e;
    *y = strtod(s, &e);
    if (*e > 0) return false;
    return true;
}

enum Sect {
    S_NONE = -1, S_TITLE, S_OPTION, S_EVAP, S_JUNC, S_OUTFALL, S_CONDUIT, S_XSECT, S_LOSS,
    S_POLLUT, S_INFLOW, S_DWF, S_PATTERN, S_TSERIES, S_REPORT, S_FILES, S_STORAGE, S_CURVES,
    S_PUMP, S_ORIFICE, S_WEIR, S_OUTLET, S_TRANSECT, S_DIVIDER, S_STREET, S_ADJUST, S_TEMP, S_SKIP, S_UNSUPPORTED
};
static const char* const kSectWords[] = {
    "[TITLE", "[OPTION", "[EVAP", "[JUNC", "[OUTFALL", "[CONDUIT", "[XSECT", "[LOSS",
    "[POLLUT", "[INFLOW", "[DWF", "[PATTERN", "[TIMESERIES", "[REPORT", "[FILES", "[STORAGE",
    "[CURVE", "[PUMP", "[ORIFICE", "[WEIR", "[OUTLET", "[TRANSECT", "[DIVIDER", "[STREET", "[ADJUST", "[TEMP", nullptr};
static const char* const kOffOnWords[] = {"OFF", "ON", nullptr};
static const char* const kOrificeTypeWords[] = {"SIDE", "BOTTOM", nullptr};
static const char* const kWeirTypeWords[] = {"TRANSVERSE", "SIDEFLOW", "V-NOTCH", "TRAPEZOIDAL",
                                             "ROADWAY", nullptr};
static const char* const kRelationWords[] = {"TABULAR", "FUNCTIONAL", "CYLINDRICAL", "CONICAL",
                                             "PARABOLIC", "PYRAMIDAL", nullptr};
static const char* const kCurveTypeWords[] = {"STORAGE", "DIVERSION", "TIDAL", "RATING", "CONTROL",
                                              "SHAPE", "WEIR", "PUMP1", "PUMP2", "PUMP3", "PUMP4",
                                              "PUMP5", nullptr};
static const char* const kTransectWords[] = {"NC", "X1", "GR", nullptr};
static const char* const kSkipWords[] = {
    "[MAP", "[COORDINATE", "[VERTICES", "[POLYGON", "[SYMBOL", "[LABEL", "[BACKDROP", "[TAG",
    "[PROFILE", nullptr};

static const char* const kFlowUnitWords[] = {"CFS", "GPM", "MGD", "CMS", "LPS", "MLD", nullptr};
static const char* const kNoYes[] = {"NO", "YES", nullptr};
static const char* const kRouteWords[] = {"NONE", "STEADY", "KINWAVE", "XKINWAVE", "DYNWAVE", nullptr};
static const char* const kOldRouteWords[] = {"NONE", "NF", "KW", "EKW", "DW", nullptr};
static const char* const kInertWords[] = {"NONE", "PARTIAL", "FULL", nullptr};
static const char* const kNormalWords[] = {"SLOPE", "FROUDE", "BOTH", "NONE", nullptr};
static const char* const kSurchargeWords[] = {"EXTRAN", "SLOT", nullptr};
static const char* const kOffsetWords[] = {"DEPTH", "ELEVATION", nullptr};
static const char* const kForceMainWords[] = {"H-W", "D-W", nullptr};
static const char* const kOutfallWords[] = {"FREE", "NORMAL", "FIXED", "TIDAL", "TIMESERIES", nullptr};
static const char* const kPatternWords[] = {"MONTHLY", "DAILY", "HOURLY", "WEEKEND", nullptr};
static const char* const kQualUnitWords[] = {"MG/L", "UG/L", "#/L", nullptr};
static const char* const kXsectWords[] = {
    "DUMMY", "CIRCULAR", "FILLED_CIRCULAR", "RECT_CLOSED", "RECT_OPEN", "TRAPEZOIDAL",
    "TRIANGULAR", "PARABOLIC", "POWER", "RECT_TRIANGULAR", "RECT_ROUND", "MODBASKETHANDLE",
    "HORIZ_ELLIPSE", "VERT_ELLIPSE", "ARCH", "EGG", "HORSESHOE", "GOTHIC", "CATENARY",
    "SEMIELLIPTICAL", "BASKETHANDLE", "SEMICIRCULAR", "IRREGULAR", "CUSTOM", "FORCE_MAIN",
    "STREET", nullptr};
// option keywords, in the reference's order (keywords.c:75-98)
enum {
    O_FLOW_UNITS, O_INFIL_MODEL, O_ROUTE_MODEL, O_START_DATE, O_START_TIME, O_END_DATE,
    O_END_TIME, O_REPORT_START_DATE, O_REPORT_START_TIME, O_SWEEP_START, O_SWEEP_END,
    O_START_DRY_DAYS, O_WET_STEP, O_DRY_STEP, O_ROUTE_STEP, O_RULE_STEP, O_REPORT_STEP,
    O_ALLOW_PONDING, O_INERT_DAMPING, O_SLOPE_WEIGHTING, O_VARIABLE_STEP, O_NORMAL_FLOW_LTD,
    O_LENGTHENING_STEP, O_MIN_SURFAREA, O_COMPATIBILITY, O_SKIP_STEADY_STATE, O_TEMPDIR,
    O_IGNORE_RAINFALL, O_FORCE_MAIN_EQN, O_LINK_OFFSETS, O_MIN_SLOPE, O_IGNORE_SNOWMELT,
    O_IGNORE_GWATER, O_IGNORE_ROUTING, O_IGNORE_QUALITY, O_MAX_TRIALS, O_HEAD_TOL,
    O_SYS_FLOW_TOL, O_LAT_FLOW_TOL, O_IGNORE_RDII, O_MIN_ROUTE_STEP, O_NUM_THREADS,
    O_SURCHARGE_METHOD
};
static const char* const kOptionWords[] = {
    "FLOW_UNITS", "INFILTRATION", "FLOW_ROUTING", "START_DATE", "START_TIME", "END_DATE",
    "END_TIME", "REPORT_START_DATE", "REPORT_START_TIME", "SWEEP_START", "SWEEP_END",
    "DRY_DAYS", "WET_STEP", "DRY_STEP", "ROUTING_STEP", "RULE_STEP", "REPORT_STEP",
    "ALLOW_PONDING", "INERTIAL_DAMPING", "SLOPE_WEIGHTING", "VARIABLE_STEP",
    "NORMAL_FLOW_LIMITED", "LENGTHENING_STEP", "MIN_SURFAREA", "COMPATIBILITY",
    "SKIP_STEADY_STATE", "TEMPDIR", "IGNORE_RAINFALL", "FORCE_MAIN_EQUATION", "LINK_OFFSETS",
    "MIN_SLOPE", "IGNORE_SNOWMELT", "IGNORE_GROUNDWATER", "IGNORE_ROUTING", "IGNORE_QUALITY",
    "MAX_TRIALS", "HEAD_TOLERANCE", "SYS_FLOW_TOL", "LAT_FLOW_TOL", "IGNORE_RDII",
    "MINIMUM_STEP", "THREADS", "SURCHARGE_METHOD", nullptr};

// ========================================================= unit conversion
// swmm5.c:105-120 (Ucf / Qcf) and UCF() swmm5.c:1378-1388
double Project::ucfLength() const { return opt.unitSystem ? 0.3048 : 1.0; }
double Project::ucfVolume() const { return opt.unitSystem ? 0.02832 : 1.0; }
double Project::ucfRainfall() const { return opt.unitSystem ? 1097280.0 : 43200.0; }
double Project::ucfEvapRate() const { return opt.unitSystem ? 26334720.0 : 1036800.0; }
double Project::ucfFlow() const
{
    static const double qcf[6] = {1.0, 448.831, 0.64632, 0.02832, 28.317, 2.4466};
    return qcf[opt.flowUnits];
}

int Project::setError(int code, const std::string& msg)
{
    if (!errorCode) {
        errorCode = code;
        errorMsg = msg;
    }
    return code;
}

int Project::addError(int code, const std::string& msg)
{
    if (!errorCode) return setError(code, msg);
    moreErrors.emplace_back(code, msg);
    return code;
}

// ============================================================ .inp reading
int Project::open(const char* path)
{
    // InpDir: directory of the input file with its trailing delimiter
    // (getAbsolutePath, swmm5.c:1571-1606)
    {
        char buf[4096];
        std::string full = (path[0] != '/' && realpath(path, buf)) ? std::string(buf) : std::string(path);
        size_t k = full.rfind('/');
        inpDir = (k == std::string::npos) ? std::string() : full.substr(0, k + 1);
    }
    if (readFile(path)) return errorCode;
    // project.c:147-181 -- run dates and durations
    opt.startDateTime = opt.startDate + opt.startTime;
    opt.endDateTime = opt.endDate + opt.endTime;
    opt.reportStart = gmax(opt.reportStartDate + opt.reportStartTime, opt.startDateTime);
    if (opt.endDateTime <= opt.startDateTime) return setError(191, "ERROR 191: simulation start date comes after ending date.");
    if (opt.endDateTime <= opt.reportStart) return setError(193, "ERROR 193: report start date comes after ending date.");
    opt.totalDuration = floor((opt.endDateTime - opt.startDateTime) * kSecPerDay);
    if ((double)opt.reportStep > opt.totalDuration) opt.reportStep = (int)opt.totalDuration;
    if ((double)opt.reportStep < opt.routeStep) return setError(195, "ERROR 195: reporting time step or duration is less than routing time step.");
    opt.totalDuration *= 1000.0;
    validate();
    return errorCode;
}

int Project::readFile(const char* path)
{
    FILE* f = fopen(path, "rb");
    if (!f) return setError(303, std::string("ERROR 303: cannot open input file ") + path);
    std::vector<char> buf;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    buf.resize((size_t)sz + 2);
    size_t got = fread(buf.data(), 1, (size_t)sz, f);
    fclose(f);
    buf[got] = '\n';
    buf[got + 1] = '\0';

    // split into lines once; each pass tokenises its own copy
    std::vector<std::pair<size_t, size_t>> lines;
    lines.reserve(got / 32 + 16);
    size_t st0 = 0;
    for (size_t i = 0; i <= got; i++)
        if (buf[i] == '\n') { lines.push_back({st0, i}); st0 = i + 1; }

    std::vector<char> work;
    std::vector<char*> tok;
    for (int pass = 1; pass <= 2; pass++) {
        int sect = S_NONE;
        for (size_t li = 0; li < lines.size(); li++) {
            size_t a = lines[li].first, b = lines[li].second;
            work.assign(buf.begin() + a, buf.begin() + b);
            work.push_back('\0');
            int nt = tokenize(work.data(), tok);
            if (nt == 0 || tok[0][0] == ';') continue;
            if (tok[0][0] == '[') {
                int s = kfind(tok[0], kSectWords);
                if (s >= 0) {
                    // input.c:210-213 -- finish the last transect
                    if (sect == S_TRANSECT && pass == 2) {
                        validateTransect(tin_.count - 1);
                        if (errorCode) return errorCode;
                    }
                    sect = s;
                    continue;
                }
                if (kfind(tok[0], kSkipWords) >= 0) { sect = S_SKIP; continue; }
                return setError(200, std::string("ERROR 200: input section ") + tok[0] +
                                          " is not supported by the MI355X dynamic-wave engine");
            }
            if (sect == S_TITLE) {
                if (pass == 2 && net.title.empty()) {
                    std::string t(buf.begin() + a, buf.begin() + b);
                    while (!t.empty() && (t.back() == '\r' || t.back() == '\n')) t.pop_back();
                    net.title = t;
                }
                continue;
            }
            if (sect == S_SKIP || sect == S_NONE) continue;
            int err = parseLine(sect, tok, pass);
            if (err) {
                if (!errorCode) {
                    char msg[512];
                    snprintf(msg, sizeof msg, "ERROR %d: input error at line %zu", err, li + 1);
                    setError(200, msg);
                }
                return errorCode;
            }
        }
        if (pass == 1) {
            // allocate per-object arrays (createObjects, project.c) -- filled in pass 2
            int nn = (int)net.nodeId.size(), nl = (int)net.linkId.size();
            net.nodeType.assign(nn, JUNCTION); net.nodeSub.assign(nn, 0); net.degree.assign(nn, 0);
            net.rptFlag.assign(nn, 0); net.invertElev.assign(nn, 0); net.initDepth.assign(nn, 0);
            net.fullDepth.assign(nn, 0); net.surDepth.assign(nn, 0); net.pondedArea.assign(nn, 0);
            net.crownElev.assign(nn, 0); net.fullVolume.assign(nn, 0); net.outfallType.assign(nn, -1);
            net.outfallFlap.assign(nn, 0); net.outfallSeries.assign(nn, -1); net.fixedStage.assign(nn, 0);
            net.stShape.assign(nn, -1); net.stCurve.assign(nn, -1); net.stA0.assign(nn, 0);
            net.stA1.assign(nn, 0); net.stA2.assign(nn, 0); net.stFEvap.assign(nn, 0);
            net.stExS.assign(nn, 0); net.stExKs.assign(nn, 0); net.stExIMD.assign(nn, 0);
            net.linkType.assign(nl, CONDUIT); net.node1.assign(nl, 0); net.node2.assign(nl, 0);
            net.hasFlapGate.assign(nl, 0); net.direction.assign(nl, 1); net.barrels.assign(nl, 1);
            net.hasLosses.assign(nl, 0); net.superCritical.assign(nl, 0); net.linkRpt.assign(nl, 0);
            for (auto* v : {&net.offset1, &net.offset2, &net.q0, &net.qLimit, &net.cLossInlet,
                            &net.cLossOutlet, &net.cLossAvg, &net.seepRate, &net.length, &net.lengthT,
                            &net.roughness, &net.modLength, &net.roughFactor, &net.slope,
                            &net.beta, &net.qMax, &net.qFull})
                v->assign(nl, 0.0);
            net.xsect.assign(nl, Xsect());
            net.ncSub.assign(nl, 0); net.ncCurve.assign(nl, -1); net.ncCanSurcharge.assign(nl, 1);
            net.ncRoadWidth.assign(nl, 0.0); net.ncRoadSurf.assign(nl, 0);
            for (auto* v : {&net.ncC1, &net.ncC2, &net.ncEndCon, &net.ncSlope, &net.ncLength,
                            &net.ncYOn, &net.ncYOff, &net.ncXMin, &net.ncXMax})
                v->assign(nl, 0.0);
            net.ncInitSetting.assign(nl, 1.0);
            for (auto& ts : net.tseries) ts.lastDate = opt.startDate + opt.startTime;  // input.c:168-171
            for (auto& p : net.patterns) { p.type = -1; p.count = 0; for (double& x : p.factor) x = 1.0; }
        }
    }
    return errorCode;
}

static int addId(std::unordered_map<std::string, int>& idx, std::vector<std::string>& ids,
                 const char* id)
{
    auto it = idx.find(id);
    if (it != idx.end()) return -1;
    int n = (int)ids.size();
    idx.emplace(id, n);
    ids.push_back(id);
    return n;
}

int Project::parseLine(int sect, std::vector<char*>& tok, int pass)
{
    int nt = (int)tok.size();
    if (pass == 1) {
        switch (sect) {
        case S_OPTION:
            if (nt < 2) return 203;
            return readOption(tok[0], tok[1]);
        case S_JUNC:
        case S_OUTFALL:
        case S_STORAGE:
        case S_DIVIDER:
            if (addId(net.nodeIndex, net.nodeId, tok[0]) < 0) return setError(207, std::string("ERROR 207: duplicate ID name ") + tok[0]);
            return 0;
        case S_STREET:
            if (net.streetIndex.count(tok[0]))
                return setError(207, std::string("ERROR 207: duplicate ID name ") + tok[0]);
            net.streetIndex.emplace(tok[0], (int)net.streets.size());
            net.streets.push_back(XTable());
            net.streets.back().id = tok[0];
            return 0;
        case S_TRANSECT:
            if (kfind(tok[0], kTransectWords) == 1 && nt >= 2) {
                if (net.transectIndex.count(tok[1]))
                    return setError(207, std::string("ERROR 207: duplicate ID name ") + tok[1]);
                net.transectIndex.emplace(tok[1], (int)net.transects.size());
                XTable t;
                t.id = tok[1];
                net.transects.push_back(t);
            }
            return 0;
        case S_CURVES:
            if (!net.curveIndex.count(tok[0])) {
                net.curveIndex.emplace(tok[0], (int)net.curves.size());
                Curve c;
                c.id = tok[0];
                net.curves.push_back(c);
            }
            return 0;
        case S_CONDUIT:
        case S_PUMP:
        case S_ORIFICE:
        case S_WEIR:
        case S_OUTLET:
            if (addId(net.linkIndex, net.linkId, tok[0]) < 0) return setError(207, std::string("ERROR 207: duplicate ID name ") + tok[0]);
            return 0;
        case S_POLLUT: {
            std::vector<std::string> ids;
            for (auto& p : net.pollut) ids.push_back(p.id);
            if (net.pollutIndex.count(tok[0])) return setError(207, std::string("ERROR 207: duplicate ID name ") + tok[0]);
            net.pollutIndex.emplace(tok[0], (int)net.pollut.size());
            Pollutant p;
            p.id = tok[0];
            net.pollut.push_back(p);
            return 0;
        }
        case S_PATTERN:
            if (!net.patternIndex.count(tok[0])) {
                net.patternIndex.emplace(tok[0], (int)net.patterns.size());
                Pattern p;
                p.id = tok[0];
                net.patterns.push_back(p);
            }
            return 0;
        case S_TSERIES:
            if (!net.tseriesIndex.count(tok[0])) {
                net.tseriesIndex.emplace(tok[0], (int)net.tseries.size());
                Tseries t;
                t.id = tok[0];
                net.tseries.push_back(t);
            }
            return 0;
        default:
            return 0;
        }
    }
    switch (sect) {
    case S_OPTION: return 0;
    case S_EVAP: return readEvap(tok);
    case S_ADJUST: return readAdjust(tok);
    case S_TEMP: return readTemperature(tok);
    case S_JUNC: return readJunction(tok);
    case S_DIVIDER: return readDivider(tok);
    case S_OUTFALL: return readOutfall(tok);
    case S_CONDUIT: return readConduit(tok);
    case S_XSECT: return readXsect(tok);
    case S_LOSS: return readLoss(tok);
    case S_POLLUT: return readPollutant(tok);
    case S_INFLOW: return readInflow(tok);
    case S_DWF: return readDwf(tok);
    case S_PATTERN: return readPattern(tok);
    case S_TSERIES: return readTimeseries(tok);
    case S_REPORT: return readReport(tok);
    case S_FILES: return readFiles(tok);
    case S_STORAGE: return readStorage(tok);
    case S_PUMP: case S_ORIFICE: case S_WEIR: case S_OUTLET: return readRegulator(sect, tok);
    case S_CURVES: return readCurve(tok);
    case S_TRANSECT: return readTransect(tok);
    case S_STREET: return readStreet(tok);
    default: return 0;
    }
}

static int hmsSeconds(double aTime)
{
    int h, m, s;
    decodeTime(aTime, &h, &m, &s);
    h += 24 * (int)aTime;
    return s + 60 * m + 3600 * h;
}

int Project::readOption(const char* s1, const char* s2)  // project.c:445-769
{
    int k = kfind(s1, kOptionWords), m;
    double t, aTime;
    if (k < 0) return 205;
    switch (k) {
    case O_FLOW_UNITS:
        m = kfind(s2, kFlowUnitWords);
        if (m < 0) return 205;
        opt.flowUnits = m;
        opt.unitSystem = (m <= MGD) ? 0 : 1;
        break;
    case O_ROUTE_MODEL:
        m = kfind(s2, kRouteWords);
        if (m < 0) m = kfind(s2, kOldRouteWords);
        if (m < 0) return 205;
        if (m == 0) opt.ignoreRouting = 1;
        else opt.routeModel = m;
        if (opt.routeModel != RM_DW || opt.ignoreRouting)
            return setError(200, "ERROR 200: only FLOW_ROUTING DYNWAVE is supported by the MI355X engine");
        break;
    case O_START_DATE: if (!strToDate(s2, &opt.startDate)) return 213; break;
    case O_START_TIME: if (!strToTime(s2, &opt.startTime)) return 213; break;
    case O_END_DATE: if (!strToDate(s2, &opt.endDate)) return 213; break;
    case O_END_TIME: if (!strToTime(s2, &opt.endTime)) return 213; break;
    case O_REPORT_START_DATE:
        if (!strToDate(s2, &opt.reportStartDate)) return 213;
        opt.haveReportStartDate = true;
        break;
    case O_REPORT_START_TIME:
        if (!strToTime(s2, &opt.reportStartTime)) return 213;
        opt.haveReportStartTime = true;
        break;
    case O_WET_STEP: case O_DRY_STEP: case O_REPORT_STEP: case O_RULE_STEP: {
        if (!strToTime(s2, &aTime)) return 213;
        int s = hmsSeconds(aTime);
        if (k == O_RULE_STEP) { if (s < 0) return 211; }
        else if (s <= 0) return 211;
        if (k == O_WET_STEP) opt.wetStep = s;
        else if (k == O_DRY_STEP) opt.dryStep = s;
        else if (k == O_REPORT_STEP) opt.reportStep = s;
        else opt.ruleStep = s;
        if (k == O_RULE_STEP && s > 0)
            return setError(200, "ERROR 200: RULE_STEP (control rules) is not supported by the MI355X engine");
        break;
    }
    case O_INERT_DAMPING:
        m = kfind(s2, kInertWords);
        if (m < 0) return 205;
        opt.inertDamping = m;
        break;
    case O_ALLOW_PONDING: case O_SLOPE_WEIGHTING: case O_SKIP_STEADY_STATE:
    case O_IGNORE_RAINFALL: case O_IGNORE_SNOWMELT: case O_IGNORE_GWATER:
    case O_IGNORE_ROUTING: case O_IGNORE_QUALITY: case O_IGNORE_RDII:
        m = kfind(s2, kNoYes);
        if (m < 0) return 205;
        if (k == O_ALLOW_PONDING) opt.allowPonding = m;
        else if (k == O_SKIP_STEADY_STATE) opt.skipSteadyState = m;
        else if (k == O_IGNORE_ROUTING) opt.ignoreRouting = m;
        else if (k == O_IGNORE_QUALITY) opt.ignoreQuality = m;
        if (opt.ignoreRouting)
            return setError(200, "ERROR 200: IGNORE_ROUTING leaves nothing for the routing engine to do");
        break;
    case O_NORMAL_FLOW_LTD:
        m = kfind(s2, kNormalWords);
        if (m < 0) return 205;
        opt.normalFlowLtd = m;
        break;
    case O_FORCE_MAIN_EQN:
        m = kfind(s2, kForceMainWords);
        if (m < 0) return 205;
        opt.forceMainEqn = m;
        break;
    case O_LINK_OFFSETS:
        m = kfind(s2, kOffsetWords);
        if (m < 0) return 205;
        opt.linkOffsetsElev = m;
        break;
    case O_ROUTE_STEP: case O_LENGTHENING_STEP:
        if (!getDouble(s2, &t)) {
            if (!strToTime(s2, &aTime)) return 211;
            t = hmsSeconds(aTime);
        }
        if (k == O_ROUTE_STEP) {
            if (t <= 0.0) return 211;
            opt.routeStep = t;
        } else {
            opt.lengtheningStep = gmax(0.0, t);
        }
        break;
    case O_MIN_ROUTE_STEP:
        if (!getDouble(s2, &opt.minRouteStep) || opt.minRouteStep < 0.0) return 211;
        break;
    case O_NUM_THREADS:
        m = atoi(s2);
        if (m < 0) return 211;
        opt.numThreads = m;
        break;
    case O_VARIABLE_STEP:
        if (!getDouble(s2, &opt.courantFactor)) return 211;
        if (opt.courantFactor < 0.0 || opt.courantFactor > 2.0) return 211;
        break;
    case O_MIN_SURFAREA:
        if (!getDouble(s2, &opt.minSurfArea) || opt.minSurfArea < 0.0) return 211;
        break;
    case O_MIN_SLOPE:
        if (!getDouble(s2, &opt.minSlope)) return 211;
        if (opt.minSlope < 0.0 || opt.minSlope >= 100) return 211;
        opt.minSlope /= 100.0;
        break;
    case O_MAX_TRIALS:
        m = atoi(s2);
        if (m < 0) return 211;
        opt.maxTrials = m;
        break;
    case O_HEAD_TOL:
        if (!getDouble(s2, &opt.headTol)) return 211;
        break;
    case O_SYS_FLOW_TOL:
        if (!getDouble(s2, &opt.sysFlowTol)) return 211;
        opt.sysFlowTol /= 100.0;
        break;
    case O_LAT_FLOW_TOL:
        if (!getDouble(s2, &opt.latFlowTol)) return 211;
        opt.latFlowTol /= 100.0;
        break;
    case O_SURCHARGE_METHOD:
        m = kfind(s2, kSurchargeWords);
        if (m < 0) return 205;
        opt.surchargeMethod = m;
        break;
    default:
        break;  // INFILTRATION, SWEEP_*, DRY_DAYS, COMPATIBILITY, TEMPDIR: no routing effect
    }
    return 0;
}

// climate_readEvapParams (climate.c:285-372): CONSTANT, MONTHLY,
// TIMESERIES, TEMPERATURE (Hargreaves, from a climate file's temperatures)
// and FILE (the climate file's pan evaporation times monthly pan
// coefficients) evaporation; the RECOVERY pattern (storage exfiltration's
// soil recovery); DRY_ONLY (runoff) is read and checked only.
int Project::readEvap(std::vector<char*>& tok)
{
    static const char* const kEvapWords[] = {"CONSTANT", "MONTHLY", "TIMESERIES", "TEMPERATURE", "FILE",
                                             "RECOVERY", "DRY_ONLY", nullptr};
    const int nt = (int)tok.size();
    const int k = kfind(tok[0], kEvapWords);
    if (k < 0) return 205;
    if (k == 5) {                                  // RECOVERY pattern
        if (nt < 2) return 203;
        auto it = net.patternIndex.find(tok[1]);
        if (it == net.patternIndex.end()) return 209;
        opt.evapRecovery = it->second;
        return 0;
    }
    if (k == 6) {                                  // DRY_ONLY YES / NO
        if (nt < 2) return 203;
        return kfind(tok[1], kNoYes) >= 0 ? 0 : 205;
    }
    opt.evapType = k;
    if (k == 3) return 0;                          // TEMPERATURE
    if (nt < 2) return k == 4 ? 0 : 203;
    if (k == 4) {                                  // FILE (v1 ... v12): monthly pan coefficients
        if (nt < 13) return 203;
        for (int i = 0; i < 12; i++)
            if (!getDouble(tok[i + 1], &opt.panCoeff[i])) return 211;
        return 0;
    }
    switch (k) {
    case 0: {                                      // CONSTANT
        double x;
        if (!getDouble(tok[1], &x)) return 211;      // any number (climate.c:335-338)
        for (double& m : opt.monthlyEvap) m = x;
        opt.evapRate = x / ucfEvapRate();
        return 0;
    }
    case 1:                                        // MONTHLY v1 ... v12
        if (nt < 13) return 203;
        for (int i = 0; i < 12; i++)
            if (!getDouble(tok[i + 1], &opt.monthlyEvap[i])) return 211;
        return 0;
    default: {                                     // TIMESERIES name
        auto it = net.tseriesIndex.find(tok[1]);
        if (it == net.tseriesIndex.end()) return 209;
        opt.evapSeries = it->second;
        return 0;
    }
    }
}

// climate_readAdjustments (climate.c:377-475): the monthly evaporation,
// temperature (temperature evaporation) and conductivity (storage
// exfiltration, conduit seepage) adjustments; RAINFALL acts on runoff only
// and is checked and ignored.  The subcatchment patterns (N-PERV, DSTORE,
// INFIL) name a subcatchment, which the routing engine's inputs never hold:
// ERR_NAME as in the reference when its lookup fails; any other keyword is
// ERR_KEYWORD
int Project::readAdjust(std::vector<char*>& tok)
{
    const int nt = (int)tok.size();
    if (nt == 1) return 0;
    static const char* const kAdjWords[] = {"TEMP", "EVAP", "RAIN", "CONDUCT", nullptr};
    const int k = kfind(tok[0], kAdjWords);
    if (k < 0) {
        if (!strcasecmp(tok[0], "N-PERV") || !strcasecmp(tok[0], "DSTORE") || !strcasecmp(tok[0], "INFIL"))
            return nt < 3 ? 203 : 209;
        return 205;
    }
    if (nt < 13) return 203;
    for (int i = 0; i < 12; i++) {
        double x;
        if (!getDouble(tok[i + 1], &x)) return 211;
        if (k == 0) opt.adjustTemp[i] = x;
        if (k == 1) opt.adjustEvap[i] = x;
        if (k == 3) opt.adjustHydcon[i] = (x <= 0.0) ? 1.0 : x;
    }
    return 0;
}

// climate_readParams (climate.c:153-281): [TEMPERATURE].  TIMESERIES and
// FILE set the temperature source (the file also the climate file, its
// start date and GHCND units); WINDSPEED FILE needs the climate file too;
// SNOWMELT carries the latitude of temperature evaporation; ADC is checked.
int Project::readTemperature(std::vector<char*>& tok)
{
    static const char* const kTempWords[] = {"TIMESERIES", "FILE", "WINDSPEED", "SNOWMELT", "ADC", nullptr};
    static const char* const kUnitWords[] = {"C10", "C", "F", nullptr};
    const int nt = (int)tok.size();
    const int k = kfind(tok[0], kTempWords);
    if (k < 0) return 205;
    switch (k) {
    case 0: {                                      // TIMESERIES name
        if (nt < 2) return 203;
        auto it = net.tseriesIndex.find(tok[1]);
        if (it == net.tseriesIndex.end()) return 209;
        opt.tempSource = 1;
        opt.tempSeries = it->second;
        return 0;
    }
    case 1: {                                      // FILE name (start) (units)
        if (nt < 2) return 203;
        opt.tempSource = 2;
        std::string fname = tok[1];
        // addAbsolutePath (swmm5.c:1620-1633)
        const bool rel = !(strchr(fname.c_str(), ':') || fname[0] == '\\' || fname[0] == '/');
        opt.climateFile = rel ? inpDir + fname : fname;
        opt.climateStart = -693594;                // NO_DATE
        if (nt > 2 && *tok[2] != '*') {
            double d;
            if (!strToDate(tok[2], &d)) return 213;
            opt.climateStart = d;
        }
        opt.climateUnits = (opt.unitSystem == 1) ? 1 : 2;
        if (nt > 3) {
            const int u = kfind(tok[3], kUnitWords);
            if (u < 0) return 205;
            opt.climateUnits = u;
        }
        return 0;
    }
    case 2:                                        // WINDSPEED FILE | MONTHLY v1 ... v12
        if (nt < 2) return 203;
        if (!strcasecmp(tok[1], "FILE")) {
            opt.windFile = true;
            return 0;
        }
        if (nt < 14) return 203;
        opt.windFile = false;
        for (int i = 0; i < 12; i++) {
            double y;
            if (!getDouble(tok[i + 2], &y)) return 211;
        }
        return 0;
    case 3: {                                      // SNOWMELT v1 ... v6
        if (nt < 7) return 203;
        double x[6];
        for (int i = 1; i < 7; i++)
            if (!getDouble(tok[i], &x[i - 1])) return 211;
        opt.snowTipm = x[1];
        opt.snowRnm = x[2];
        opt.tempElev = x[3] / ucfLength();
        opt.anglat = x[4];
        opt.dtlong = x[5] / 60.0;
        return 0;
    }
    default: {                                     // ADC IMPERV/PERV v1 ... v10
        if (nt < 12) return 203;
        static const char* const kAdcWords[] = {"IMPERV", "PERV", nullptr};
        if (kfind(tok[1], kAdcWords) < 0) return 205;
        for (int j = 0; j < 10; j++) {
            double y;
            if (!getDouble(tok[j + 2], &y) || y < 0.0 || y > 1.0) return 211;
        }
        return 0;
    }
    }
}

// divider_readParams (node.c:1124-1212).  Under dynamic wave a flow divider
// routes as a junction (its diversion rule serves kinematic-wave routing
// only); its parameters are read and validated as the reference does.
int Project::readDivider(std::vector<char*>& tok)
{
    int nt = (int)tok.size();
    if (nt < 4) return 203;
    int j = net.nodeIndex.at(tok[0]);
    double x[11];
    if (!getDouble(tok[1], &x[0])) return 211;
    for (int i = 1; i < 11; i++) x[i] = 0.0;
    if (strlen(tok[2]) == 0 || strcmp(tok[2], "*") == 0) x[1] = -1.0;
    else {
        auto it = net.linkIndex.find(tok[2]);
        if (it == net.linkIndex.end()) return 209;
        x[1] = it->second;
    }
    static const char* const kDividerWords[] = {"CUTOFF", "TABULAR", "WEIR", "OVERFLOW", nullptr};
    int n = 4;
    int m1 = kfind(tok[3], kDividerWords);
    if (m1 < 0) return 205;
    x[2] = m1;
    x[3] = -1;
    if (m1 == 1) {                                   // TABULAR: diversion curve
        if (nt < 5) return 203;
        auto it = net.curveIndex.find(tok[4]);
        if (it == net.curveIndex.end()) return 209;
        x[3] = it->second;
        n = 5;
    }
    if (m1 == 0) {                                   // CUTOFF: cutoff flow
        if (nt < 5) return 203;
        if (!getDouble(tok[4], &x[4])) return 211;
        n = 5;
    }
    if (m1 == 2) {                                   // WEIR: qMin, dhMax, cWeir
        if (nt < 7) return 203;
        for (int i = 4; i < 7; i++)
            if (!getDouble(tok[i], &x[i])) return 211;
        n = 7;
    }
    if (m1 == 3) n = 4;
    int m = 7;
    for (int i = n; i < nt && m < 11; i++) {
        if (!getDouble(tok[i], &x[m])) return 211;
        m++;
    }
    double u = ucfLength();
    net.nodeType[j] = DIVIDER;
    net.invertElev[j] = x[0] / u;
    net.crownElev[j] = net.invertElev[j];
    net.fullDepth[j] = x[7] / u;
    net.initDepth[j] = x[8] / u;
    net.surDepth[j] = x[9] / u;
    net.pondedArea[j] = x[10] / (u * u);
    Divider dv;
    dv.node = j;
    dv.link = (int)x[1];
    dv.type = m1;
    dv.qMin = x[4] / ucfFlow();
    dv.dhMax = x[5];
    dv.cWeir = x[6];
    net.dividers.push_back(dv);
    return 0;
}

int Project::readJunction(std::vector<char*>& tok)  // node.c:606-648, 125-196
{
    int nt = (int)tok.size();
    if (nt < 2) return 203;
    int j = net.nodeIndex.at(tok[0]);
    double x[6];
    for (int i = 1; i <= 5; i++) {
        x[i - 1] = 0.0;
        if (i < nt && !getDouble(tok[i], &x[i - 1])) return 211;
    }
    for (int i = 1; i <= 4; i++)
        if (x[i] < 0.0) return 211;
    double u = ucfLength();
    net.nodeType[j] = JUNCTION;
    net.invertElev[j] = x[0] / u;
    net.crownElev[j] = net.invertElev[j];
    net.fullDepth[j] = x[1] / u;
    net.initDepth[j] = x[2] / u;
    net.surDepth[j] = x[3] / u;
    net.pondedArea[j] = x[4] / (u * u);
    return 0;
}

// storage_readParams (node.c:654-809):
//   id elev maxDepth initDepth shape a1 a2 a0 | TABULAR curve  [surDepth [fEvap [seepage]]]
int Project::readStorage(std::vector<char*>& tok)
{
    int nt = (int)tok.size();
    if (nt < 6) return 203;
    int j = net.nodeIndex.at(tok[0]);
    double x[3];
    for (int i = 1; i <= 3; i++)
        if (!getDouble(tok[i], &x[i - 1])) return 211;
    int m = kfind(tok[4], kRelationWords);
    if (m < 0) return 205;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, y[3] = {0, 0, 0};
    int curve = -1, n;
    if (m == ST_TABULAR) {
        auto it = net.curveIndex.find(tok[5]);
        if (it == net.curveIndex.end()) return 209;
        curve = it->second;
        n = 6;
    } else {
        if (nt < 8) return 203;
        for (int i = 5; i <= 7; i++)
            if (!getDouble(tok[i], &y[i - 5])) return 211;
        n = 8;
    }
    switch (m) {
    case ST_FUNCTIONAL:
        if (y[2] < 0.0) return 211;
        break;
    case ST_CYLINDRICAL: case ST_CONICAL: case ST_PARABOLOID: case ST_PYRAMIDAL:
        if (y[0] <= 0.0 || y[1] <= 0.0 || y[2] < 0.0) return 211;
        break;
    }
    if (m == ST_PARABOLOID && y[2] == 0.0) return 211;
    const double PI = 3.141592654;
    double A, B, Z, L, W;
    switch (m) {
    case ST_FUNCTIONAL: a1 = y[0]; a2 = y[1]; a0 = y[2]; break;
    case ST_CYLINDRICAL:
        A = y[0] / 2.; B = y[1] / 2.;
        a1 = 0.0; a2 = 0.0; a0 = PI * A * B;
        break;
    case ST_CONICAL:
        A = y[0] / 2.; B = y[1] / 2.; Z = y[2];
        a1 = 2.0 * PI * B * Z; a2 = PI * B / A * Z * Z; a0 = PI * A * B;
        break;
    case ST_PARABOLOID:
        A = y[0] / 2.; B = y[1] / 2.; Z = y[2];
        a1 = PI * A * B / Z; a2 = 0.0; a0 = 0.0;
        break;
    case ST_PYRAMIDAL:
        L = y[0]; W = y[1]; Z = y[2];
        a1 = 2.0 * (L + W) * Z; a2 = 4.0 * Z * Z; a0 = L * W;
        break;
    }
    double surDepth = 0.0, fEvap = 0.0;
    if (nt > n) { if (!getDouble(tok[n], &surDepth)) return 211; n++; }
    if (nt > n) { if (!getDouble(tok[n], &fEvap)) return 211; n++; }
    double ex[3] = {0.0, 0.0, 0.0};     // suction head, Ksat, IMDmax (user units)
    if (nt > n) {                       // exfil_readStorageParams (exfil.c:34-70)
        if (nt == n + 1) { if (!getDouble(tok[n], &ex[1])) return 211; }
        else if (nt < n + 3) return 203;
        else {
            for (int i = 0; i < 3; i++) if (!getDouble(tok[n + i], &ex[i])) return 211;
        }
        if (ex[1] != 0.0) {
            // createStorageExfil -> grnampt_setParams (infil.c:574-593)
            if (ex[0] < 0.0 || ex[1] <= 0.0 || ex[2] < 0.0 || ex[2] > 1.0) return 211;
            // exfil_initState (exfil.c:83-150) leaves a PARABOLIC unit's
            // bottom and bank geometry unset in the reference (undefined)
            if (m == ST_PARABOLOID)
                return setError(200, "ERROR 200: seepage from a PARABOLIC storage unit is not supported "
                                     "by the MI355X engine (its exfiltration geometry is undefined in SWMM 5.2)");
        }
    }
    double u = ucfLength();
    net.nodeType[j] = STORAGE;
    net.invertElev[j] = x[0] / u;
    net.crownElev[j] = net.invertElev[j];
    net.fullDepth[j] = x[1] / u;
    net.initDepth[j] = x[2] / u;
    net.surDepth[j] = surDepth / u;
    net.pondedArea[j] = 0.0;
    net.stShape[j] = m;
    net.stCurve[j] = curve;
    net.stA0[j] = a0;
    net.stA1[j] = a1;
    net.stA2[j] = a2;
    net.stFEvap[j] = fEvap;
    if (ex[1] != 0.0) {                 // grnampt_setParams' conversions
        net.stExS[j] = ex[0] / (opt.unitSystem ? 304.8 : 12.0);   // UCF(RAINDEPTH)
        net.stExKs[j] = ex[1] / ucfRainfall();
        net.stExIMD[j] = ex[2];
    }
    net.nStorage++;
    return 0;
}

// table_readCurve (table.c:67-109): first line carries the curve type
int Project::readCurve(std::vector<char*>& tok)
{
    int nt = (int)tok.size();
    if (nt < 2) return 203;
    auto it = net.curveIndex.find(tok[0]);
    if (it == net.curveIndex.end()) return 209;
    Curve& c = net.curves[it->second];
    int k1 = 1;
    if (c.type < 0) {
        int m = kfind(tok[1], kCurveTypeWords);
        if (m < 0) return 205;
        c.type = m;
        if (nt == 2) return 0;
        k1 = 2;
    }
    for (int k = k1; k < nt; k += 2) {
        if (k + 1 >= nt) return 203;
        double x, y;
        if (!getDouble(tok[k], &x) || !getDouble(tok[k + 1], &y)) return 211;
        c.x.push_back(x);
        c.y.push_back(y);
    }
    return 0;
}

// ======================================================== irregular sections
// transect_readParams (transect.c:105-190): NC / X1 / GR lines, HEC-2 format
int Project::readTransect(std::vector<char*>& tok)
{
    int nt = (int)tok.size();
    TransectInput& T = tin_;
    int k = kfind(tok[0], kTransectWords);
    if (k < 0) return 205;
    double u = ucfLength();
    if (k == 0) {                                       // NC nLeft nRight nChannel
        validateTransect(T.count - 1);
        if (errorCode) return errorCode;
        if (nt < 4) return 203;
        double n[4];
        for (int i = 1; i <= 3; i++)
            if (!getDouble(tok[i], &n[i])) return 211;
        for (int i = 1; i <= 3; i++)                    // setManning transect.c:312-330
            if (n[i] < 0.0) return 211;
        if (n[1] > 0.0) T.nLeft = n[1];
        if (n[2] > 0.0) T.nRight = n[2];
        if (n[3] > 0.0) T.nChannel = n[3];
        if (T.nLeft == 0.0) T.nLeft = T.nChannel;
        if (T.nRight == 0.0) T.nRight = T.nChannel;
        return 0;
    }
    if (k == 1) {                                       // X1 name nSta xLeft xRight 0 0 0 lFactor xFactor yFactor
        if (nt < 10) return 203;
        auto it = net.transectIndex.find(tok[1]);
        if (it == net.transectIndex.end()) return 209;
        double x[10];
        for (int i = 2; i < 10; i++)
            if (!getDouble(tok[i], &x[i])) return 211;
        int idx = T.count;
        T.count = idx + 1;
        if (idx < 0 || idx >= (int)net.transects.size()) return 211;   // setParams transect.c:334-356
        T.xLeft = x[3] / u;
        T.xRight = x[4] / u;
        T.lFactor = x[7];
        if (T.lFactor == 0.0) T.lFactor = 1.0;
        T.xFactor = x[8];
        if (T.xFactor == 0.0) T.xFactor = 1.0;
        T.xLeft *= T.xFactor;
        T.xRight *= T.xFactor;
        T.yFactor = x[9] / u;
        T.nStations = 0;
        return 0;
    }
    if ((nt - 1) % 2 > 0) return 203;                   // GR elev station ...
    for (int i = 1; i < nt; i += 2) {
        double y, x;
        if (!getDouble(tok[i], &y)) return 211;
        if (!getDouble(tok[i + 1], &x)) return 211;
        if (T.nStations < 0) return 219;                // addStation transect.c:360-384
        T.nStations++;
        if (T.nStations >= 1500) continue;
        T.station[T.nStations] = x * T.xFactor / u;
        T.elev[T.nStations] = (y + T.yFactor) / u;
        if (T.nStations > 1 && T.station[T.nStations] < T.station[T.nStations - 1]) return 221;
    }
    return 0;
}

namespace {
// the transect under construction (transect.c's file-scope arrays)
struct Slices {
    const std::vector<double>& st;
    const std::vector<double>& el;
    int n;
    double nLeft, nRight, nChannel, xLeft, xRight;
};
// getFlow (transect.c:519-566)
double sliceFlow(const Slices& S, int k, double a, double wp, bool findFlow)
{
    if (!findFlow) {
        if (k == S.n - 1) findFlow = true;
        else if (S.st[k] == S.xLeft) {
            if (S.nLeft != S.nChannel && S.st[k] != S.st[k - 1]) findFlow = true;
        } else if (S.st[k] == S.xRight) {
            if (S.nRight != S.nChannel && S.st[k] != S.st[k + 1]) findFlow = true;
        }
    }
    if (findFlow) {
        double n = S.nChannel;
        if (S.st[k - 1] < S.xLeft) n = S.nLeft;
        if (S.st[k] > S.xRight) n = S.nRight;
        return kPhi / n * a * pow(a / wp, 2. / 3.);
    }
    return 0.0;
}
// createTables / getGeometry / getSliceGeom / setMaxSectionFactor
// (transect.c:264-308, 388-515, 570-592)
void transectTables(XTable& t, const Slices& S, double ymin, double ymax)
{
    int n = t.nTbl;
    t.area.assign(n, 0.0);
    t.hrad.assign(n, 0.0);
    t.width.assign(n, 0.0);
    t.yFull = ymax - ymin;
    t.wMax = 0.0;
    double dy = (ymax - ymin) / ((double)n - 1), y = ymin;
    for (int i = 1; i < n; i++) {
        y += dy;
        double wpSum = 0.0, aSum = 0.0, qSum = 0.0;
        for (int k = 1; k <= S.n; k++) {
            double yhi, ylo;
            if (S.el[k - 1] >= S.el[k]) { yhi = S.el[k - 1]; ylo = S.el[k]; }
            else { yhi = S.el[k]; ylo = S.el[k - 1]; }
            if (ylo >= y) continue;
            double width = fabs(S.st[k] - S.st[k - 1]);
            double w = width, wp = sqrt(width * width + (yhi - ylo) * (yhi - ylo)), a = 0.0;
            if (y > yhi) a = width * ((y - yhi) + (y - ylo)) / 2.0;
            else if (yhi > ylo) {
                double ratio = (y - ylo) / (yhi - ylo);
                a = width * (yhi - ylo) / 2.0 * ratio * ratio;
                w *= ratio;
                wp *= ratio;
            }
            wpSum += wp;
            aSum += a;
            t.area[i] += a;
            t.width[i] += w;
            double q = sliceFlow(S, k, aSum, wpSum, S.el[k] >= y);
            if (q > 0.0) {
                qSum += q;
                aSum = 0.0;
                wpSum = 0.0;
            }
        }
        aSum = t.area[i];
        if (aSum == 0.0) t.hrad[i] = t.hrad[i - 1];
        else t.hrad[i] = pow(qSum * S.nChannel / 1.49 / aSum, 1.5);
    }
    t.aMax = 0.0;
    t.sMax = 0.0;
    for (int i = 1; i < n; i++) {
        double sf = t.area[i] * pow(t.hrad[i], 2. / 3.);
        if (sf > t.sMax) { t.sMax = sf; t.aMax = t.area[i]; }
    }
    int nLast = n - 1;
    t.aFull = t.area[nLast];
    t.rFull = t.hrad[nLast];
    t.wMax = t.width[nLast];
    for (int i = 1; i <= nLast; i++) {
        t.area[i] /= t.aFull;
        t.hrad[i] /= t.rFull;
        t.width[i] /= t.wMax;
    }
    t.width[0] = t.width[1];
}

// shape.c:42-330 -- geometry tables of a custom shape curve (relative
// height vs relative width)
bool shapeTables(XTable& t, const Curve& c)
{
    size_t next = 0;
    auto nextEntry = [&](double* x, double* y) {
        if (next >= c.x.size()) return false;
        *x = c.x[next];
        *y = c.y[next];
        next++;
        return true;
    };
    double Atotal = 0.0, Ptotal = 0.0;
    auto area = [](double y, double w, double y1, double w1) {
        double wMin, wMax;
        if (w > w1) { wMin = w1; wMax = w; } else { wMin = w; wMax = w1; }
        return (wMin + (wMax - wMin) / 2.0) * (y - y1);
    };
    auto perim = [](double y, double w, double y1, double w1) {
        double dy = y - y1, dw = fabs(w - w1) / 2.0;
        return 2.0 * sqrt(dy * dy + dw * dw);
    };
    double y1, w1, y2, w2;
    if (!nextEntry(&y1, &w1)) return false;
    if (y1 < 0.0 || y1 >= 1.0 || w1 < 0.0) return false;
    double wMax = w1;
    if (y1 != 0.0) {
        y2 = y1; w2 = w1; y1 = 0.0; w1 = 0.0;
    } else {
        if (!nextEntry(&y2, &w2)) return false;
        if (y2 < y1 || w2 < 0.0) return false;
        if (y2 > 1.0) y2 = 1.0;
        if (w2 > wMax) wMax = w2;
    }
    t.nTbl = 51;
    int n = t.nTbl - 1;
    double dy = 1.0 / (double)(n);
    t.area.assign(t.nTbl, 0.0);
    t.hrad.assign(t.nTbl, 0.0);
    t.width.assign(t.nTbl, 0.0);
    t.width[0] = w1;
    Ptotal = w1;
    Atotal = 0.0;
    double y = 0.0, w = w1;
    for (int i = 1; i <= n; i++) {
        double yLast = y, wLast = w;
        y = y + dy;
        if (fabs(y - 1.0) < 1.E-6) y = 1.0;
        if (y > y2) {                                     // getNextInterval shape.c:270-310
            while (y > y2) {
                if (y2 > yLast) {
                    Atotal += area(y2, w2, yLast, wLast);
                    Ptotal += perim(y2, w2, yLast, wLast);
                    yLast = y2;
                    wLast = w2;
                }
                y1 = y2;
                w1 = w2;
                if (!nextEntry(&y2, &w2)) { y2 = 1.0; break; }
                if (w2 > wMax) wMax = w2;
                if (y2 < y1 || w2 < 0.0) return false;
                if (y2 > 1.0) y2 = 1.0;
            }
            yLast = y1;
            wLast = w1;
        }
        w = (y2 == y1) ? w2 : w1 + (y - y1) / (y2 - y1) * (w2 - w1);
        Atotal += area(y, w, yLast, wLast);
        Ptotal += perim(y, w, yLast, wLast);
        if (y == 1.0) Ptotal += w2;
        t.width[i] = w;
        t.area[i] = Atotal;
        t.hrad[i] = (Ptotal > 0.0) ? Atotal / Ptotal : 0.0;
    }
    t.aFull = t.area[n];
    t.rFull = t.hrad[n];
    t.wMax = wMax;
    t.sMax = 0.0;
    t.aMax = 0.0;
    for (int i = 1; i <= n; i++) {
        double sf = t.area[i] * pow(t.hrad[i], 2. / 3.);
        if (sf > t.sMax) { t.sMax = sf; t.aMax = t.area[i]; }
    }
    if (t.aFull == 0.0 || t.rFull == 0.0 || t.wMax == 0.0) return false;
    for (int i = 0; i <= n; i++) {
        t.area[i] /= t.aFull;
        t.hrad[i] /= t.rFull;
        t.width[i] /= t.wMax;
    }
    return true;
}
}  // namespace

// street_readParams (street.c:58-137) and transect_createStreetTransect
// (transect.c:596-680), which builds the street's transect in the transect
// module's shared arrays and roughness state
int Project::readStreet(std::vector<char*>& tok)
{
    int nt = (int)tok.size();
    if (nt < 5) return 203;
    auto it = net.streetIndex.find(tok[0]);
    if (it == net.streetIndex.end()) return 209;
    double x[11];
    for (int k = 0; k <= 10; k++) x[k] = 0.0;
    for (int k = 1; k <= 4; k++)
        if (!getDouble(tok[k], &x[k]) || x[k] <= 0.0) return 211;
    if (nt > 5 && (!getDouble(tok[5], &x[5]) || x[5] < 0.0)) return 211;
    if (nt > 6 && (!getDouble(tok[6], &x[6]) || x[6] < 0.0)) return 211;
    int sides = 2;
    if (nt > 7) {
        char* e = nullptr;
        long v = strtol(tok[7], &e, 10);
        if (!e || *e || v < 1 || v > 2) return 211;
        sides = (int)v;
    }
    if (nt > 8) {
        if (!getDouble(tok[8], &x[8]) || x[8] < 0.0) return 211;
        if (x[8] > 0.0) {
            if (nt < 11) return 203;
            for (int k = 9; k <= 10; k++)
                if (!getDouble(tok[k], &x[k]) || x[k] <= 0.0) return 211;
        }
    }
    double u = ucfLength();
    double width = x[1] / u, curbHeight = x[2] / u, slope = x[3] / 100.0, roughness = x[4];
    double gutterDepression = x[5] / u, gutterWidth = x[6] / u;
    double backWidth = x[8] / u, backSlope = x[9] / 100.0, backRoughness = x[10];
    TransectInput& T = tin_;
    double ymin = 0.0;
    double w1 = backWidth, w2 = gutterWidth, w3 = width, w4 = w3 - w2;
    double y3 = gutterDepression + slope * w2;
    double y1 = curbHeight + gutterDepression;
    double ymax = backSlope * backWidth + y1;
    double y4 = y3 + slope * w4;
    ymax = gmax(ymax, y4);
    T.station[0] = 0.0; T.elev[0] = ymax;
    T.station[1] = w1; T.elev[1] = y1;
    T.station[2] = w1; T.elev[2] = 0.0;
    T.station[3] = w1 + w2; T.elev[3] = y3;
    T.station[4] = w1 + w3; T.elev[4] = y4;
    if (sides == 1) {
        T.station[5] = T.station[4]; T.elev[5] = ymax;
        T.nStations = 5;
    } else {
        T.station[5] = T.station[4] + w4; T.elev[5] = y3;
        T.station[6] = T.station[5] + w2; T.elev[6] = 0.0;
        T.station[7] = T.station[6]; T.elev[7] = y1;
        T.station[8] = T.station[7] + w1; T.elev[8] = ymax;
        T.nStations = 8;
    }
    T.nChannel = roughness;
    if (backWidth == 0.0) {
        T.nLeft = T.nChannel;
        T.nRight = T.nChannel;
        T.xLeft = T.station[0];
        T.xRight = T.station[T.nStations];
    } else {
        T.nLeft = backRoughness;
        T.nRight = T.nLeft;
        T.xLeft = T.station[1];
        T.xRight = (sides == 2) ? T.station[T.nStations - 1] : T.station[T.nStations];
    }
    XTable& t = net.streets[it->second];
    t.nTbl = 51;
    t.lengthFactor = 0.0;                             // never set for streets (calloc)
    Slices S{T.station, T.elev, T.nStations, T.nLeft, T.nRight, T.nChannel, T.xLeft, T.xRight};
    transectTables(t, S, ymin, ymax);
    t.roughness = roughness;
    t.valid = true;
    return 0;
}

// transect_validate (transect.c:194-260)
void Project::validateTransect(int j)
{
    TransectInput& T = tin_;
    double oldNchannel = T.nChannel;
    if (j < 0 || j >= (int)net.transects.size()) return;
    XTable& t = net.transects[j];
    const std::string id = t.id;
    if (T.nStations < 2) { setError(223, "ERROR 223: transect " + id + " has too few stations."); return; }
    if (T.nStations >= 1500) { setError(225, "ERROR 225: transect " + id + " has too many stations."); return; }
    if (T.nChannel <= 0.0) { setError(227, "ERROR 227: transect " + id + " has no Manning's N."); return; }
    if (T.xLeft > T.xRight) { setError(229, "ERROR 229: transect " + id + " has invalid overbank locations."); return; }
    T.nChannel = T.nChannel * sqrt(T.lFactor);
    t.lengthFactor = T.lFactor;
    double ymax = T.elev[1], ymin = T.elev[1];
    for (int i = 2; i <= T.nStations; i++) {
        ymax = gmax(T.elev[i], ymax);
        ymin = gmin(T.elev[i], ymin);
    }
    if (ymin >= ymax) { setError(231, "ERROR 231: transect " + id + " has no depth."); return; }
    T.station[0] = T.station[1];
    T.elev[0] = ymax;
    T.nStations++;
    T.station[T.nStations] = T.station[T.nStations - 1];
    T.elev[T.nStations] = T.elev[0];
    t.nTbl = 51;
    Slices S{T.station, T.elev, T.nStations, T.nLeft, T.nRight, T.nChannel, T.xLeft, T.xRight};
    transectTables(t, S, ymin, ymax);
    t.roughness = oldNchannel;
    t.valid = true;
}

// shape curves (project.c:220-231) and the device table blocks of every
// transect and shape: [n][A n][W n][R n] (xsect.h tabDesc)
void Project::buildXTables()
{
    net.curveShape.assign(net.curves.size(), -1);
    net.shapes.clear();
    for (size_t i = 0; i < net.curves.size(); i++) {
        if (net.curves[i].type != CV_SHAPE) continue;
        XTable t;
        t.id = net.curves[i].id;
        net.curveShape[i] = (int)net.shapes.size();
        if (!shapeTables(t, net.curves[i])) {
            setError(171, "ERROR 171: Curve " + net.curves[i].id + " has invalid or out of sequence data.");
            return;
        }
        t.valid = true;
        net.shapes.push_back(t);
    }
    net.xTab.clear();
    for (auto* v : {&net.transects, &net.shapes, &net.streets})
        for (XTable& t : *v) {
            if (t.nTbl <= 0) continue;
            t.blockOff = (int)net.xTab.size();
            net.xTab.push_back((double)t.nTbl);
            net.xTab.insert(net.xTab.end(), t.area.begin(), t.area.end());
            net.xTab.insert(net.xTab.end(), t.width.begin(), t.width.end());
            net.xTab.insert(net.xTab.end(), t.hrad.begin(), t.hrad.end());
        }
}

int Project::readOutfall(std::vector<char*>& tok)  // node.c:1333-1409
{
    int nt = (int)tok.size();
    if (nt < 3) return 203;
    int j = net.nodeIndex.at(tok[0]);
    double elev;
    if (!getDouble(tok[1], &elev)) return 211;
    int i = kfind(tok[2], kOutfallWords);
    if (i < 0) return 205;
    double stage = 0.0;
    int series = -1, flap = 0, n = 4;
    if (i >= O_FIXED) {
        if (nt < 4) return 203;
        n = 5;
        if (i == O_FIXED) {
            if (!getDouble(tok[3], &stage)) return 211;
        } else if (i == O_TSERIES) {
            auto it = net.tseriesIndex.find(tok[3]);
            if (it == net.tseriesIndex.end()) return 209;
            series = it->second;
        } else {                                    // TIDAL: the tide curve (node.c:1380-1384)
            auto it = net.curveIndex.find(tok[3]);
            if (it == net.curveIndex.end()) return 209;
            series = it->second;
        }
    }
    if (nt == n) {
        int m = kfind(tok[n - 1], kNoYes);
        if (m < 0) return 205;
        flap = m;
    }
    if (nt == n + 1)
        return setError(200, "ERROR 200: outfalls routed to subcatchments are not supported");
    double u = ucfLength();
    net.nodeType[j] = OUTFALL;
    net.invertElev[j] = elev / u;
    net.crownElev[j] = net.invertElev[j];
    net.outfallType[j] = i;
    net.fixedStage[j] = stage / u;
    net.outfallSeries[j] = series;
    net.outfallFlap[j] = flap;
    return 0;
}

int Project::readConduit(std::vector<char*>& tok)  // link.c:933-988, 315-399
{
    int nt = (int)tok.size();
    if (nt < 7) return 203;
    int j = net.linkIndex.at(tok[0]);
    auto a = net.nodeIndex.find(tok[1]);
    auto b = net.nodeIndex.find(tok[2]);
    if (a == net.nodeIndex.end() || b == net.nodeIndex.end()) return 209;
    double x[6];
    if (!getDouble(tok[3], &x[0])) return 211;
    if (!getDouble(tok[4], &x[1])) return 211;
    if (opt.linkOffsetsElev && *tok[5] == '*') x[2] = kMissing;
    else if (!getDouble(tok[5], &x[2])) return 211;
    if (opt.linkOffsetsElev && *tok[6] == '*') x[3] = kMissing;
    else if (!getDouble(tok[6], &x[3])) return 211;
    x[4] = 0.0;
    if (nt >= 8 && !getDouble(tok[7], &x[4])) return 211;
    x[5] = 0.0;
    if (nt >= 9 && !getDouble(tok[8], &x[5])) return 211;
    double u = ucfLength(), uq = ucfFlow();
    net.node1[j] = a->second;
    net.node2[j] = b->second;
    net.linkType[j] = CONDUIT;
    net.length[j] = x[0] / u;
    net.modLength[j] = net.length[j];
    net.roughness[j] = x[1];
    net.offset1[j] = x[2] / u;
    net.offset2[j] = x[3] / u;
    net.q0[j] = x[4] / uq;
    net.qLimit[j] = x[5] / uq;
    net.hasFlapGate[j] = 0;
    net.direction[j] = 1;
    return 0;
}

// pump_readParams / orifice_readParams / weir_readParams / outlet_readParams
// (link.c:1406-1469, 1641-1692, 2042-2097, 2520-2596) + link_setParams
int Project::readRegulator(int sect, std::vector<char*>& tok)
{
    int nt = (int)tok.size();
    if (nt < 3) return 203;
    int j = net.linkIndex.at(tok[0]);
    auto a = net.nodeIndex.find(tok[1]);
    auto b = net.nodeIndex.find(tok[2]);
    if (a == net.nodeIndex.end() || b == net.nodeIndex.end()) return 209;
    double u = ucfLength();
    auto curveOf = [&](const char* t) {
        auto it = net.curveIndex.find(t);
        return it == net.curveIndex.end() ? -2 : it->second;
    };
    net.node1[j] = a->second;
    net.node2[j] = b->second;
    net.offset1[j] = net.offset2[j] = 0.0;
    net.q0[j] = 0.0;
    net.qFull[j] = 0.0;
    net.hasFlapGate[j] = 0;
    net.qLimit[j] = 0.0;
    net.direction[j] = 1;
    net.barrels[j] = 0;                  // no Conduit record
    net.nNC++;
    switch (sect) {
    case S_PUMP: {
        int curve = -1;
        if (nt >= 4 && strcmp(tok[3], "*")) {
            curve = curveOf(tok[3]);
            if (curve < 0) return 209;
        }
        double init = 1.0, yOn = 0.0, yOff = 0.0;
        if (nt >= 5) {
            int m = kfind(tok[4], kOffOnWords);
            if (m < 0) return 205;
            init = m;
        }
        if (nt >= 6 && (!getDouble(tok[5], &yOn) || yOn < 0.0)) return 211;
        if (nt >= 7 && (!getDouble(tok[6], &yOff) || yOff < 0.0)) return 211;
        net.linkType[j] = PUMP;
        net.ncCurve[j] = curve;
        net.ncInitSetting[j] = init;
        net.ncYOn[j] = yOn / u;
        net.ncYOff[j] = yOff / u;
        net.xsect[j].type = -1;               // pumps have no cross section
        net.xsect[j].yFull = 0.0;
        net.nPumps++;
        return 0;
    }
    case S_ORIFICE: {
        if (nt < 6) return 203;
        int m = kfind(tok[3], kOrificeTypeWords);
        if (m < 0) return 205;
        double crest, cd, orate = 0.0;
        if (opt.linkOffsetsElev && *tok[4] == '*') crest = kMissing;
        else if (!getDouble(tok[4], &crest)) return 211;
        if (!getDouble(tok[5], &cd) || cd < 0.0) return 211;
        int flap = 0;
        if (nt >= 7) { flap = kfind(tok[6], kNoYes); if (flap < 0) return 205; }
        if (nt >= 8 && (!getDouble(tok[7], &orate) || orate < 0.0)) return 211;
        net.linkType[j] = ORIFICE;
        net.ncSub[j] = m;
        net.offset1[j] = crest <= kMissing ? crest : crest / u;
        net.offset2[j] = net.offset1[j];
        net.ncC1[j] = cd;
        net.hasFlapGate[j] = flap > 0;
        net.ncC2[j] = orate * 3600.0;
        return 0;
    }
    case S_WEIR: {
        if (nt < 6) return 203;
        int m = kfind(tok[3], kWeirTypeWords);
        if (m < 0) return 205;
        double crest, cd1, endCon = 0.0, cd2 = 0.0;
        if (opt.linkOffsetsElev && *tok[4] == '*') crest = kMissing;
        else if (!getDouble(tok[4], &crest)) return 211;
        if (!getDouble(tok[5], &cd1) || cd1 < 0.0) return 211;
        int flap = 0, surch = 1, cdCurve = -1;
        if (nt >= 7 && *tok[6] != '*') { flap = kfind(tok[6], kNoYes); if (flap < 0) return 205; }
        if (nt >= 8 && *tok[7] != '*' && (!getDouble(tok[7], &endCon) || endCon < 0.0)) return 211;
        if (nt >= 9 && *tok[8] != '*' && (!getDouble(tok[8], &cd2) || cd2 < 0.0)) return 211;
        if (nt >= 10 && *tok[9] != '*') { surch = kfind(tok[9], kNoYes); if (surch < 0) return 205; }
        double roadWidth = 0.0;
        int roadSurf = 0;
        if (m == WR_ROADWAY) {                            // link.c:2074-2086
            if (nt >= 11 && (!getDouble(tok[10], &roadWidth) || roadWidth < 0.0)) return 211;
            if (nt >= 12) {
                if (strcasecmp(tok[11], "PAVED") == 0) roadSurf = 1;
                else if (strcasecmp(tok[11], "GRAVEL") == 0) roadSurf = 2;
            }
        }
        if (nt >= 13 && *tok[12] != '*') { cdCurve = curveOf(tok[12]); if (cdCurve < 0) return 209; }
        net.ncRoadWidth[j] = roadWidth / u;
        net.ncRoadSurf[j] = roadSurf;
        net.linkType[j] = WEIR;
        net.ncSub[j] = m;
        net.offset1[j] = crest <= kMissing ? crest : crest / u;
        net.offset2[j] = net.offset1[j];
        net.ncC1[j] = cd1;
        net.hasFlapGate[j] = flap > 0;
        net.ncEndCon[j] = endCon;
        net.ncC2[j] = cd2;
        net.ncCanSurcharge[j] = surch;
        net.ncCurve[j] = cdCurve;
        return 0;
    }
    case S_OUTLET: {
        if (nt < 6) return 203;
        double crest;
        if (opt.linkOffsetsElev && *tok[3] == '*') crest = kMissing;
        else {
            if (!getDouble(tok[3], &crest)) return 211;
            if (!opt.linkOffsetsElev && crest < 0.0) crest = 0.0;
        }
        std::string rel = tok[4];
        int m = kfind(rel.c_str(), kRelationWords);
        if (m < 0) return 205;
        int ctype = 0;                        // NODE_DEPTH unless "/HEAD"
        size_t sl = rel.find('/');
        if (sl != std::string::npos) {
            std::string q = rel.substr(sl + 1);
            for (auto& ch : q) ch = (char)toupper((unsigned char)ch);
            if (q == "HEAD") ctype = 1;
        }
        double coeff = 0.0, expon = 0.0;
        int curve = -1, n;
        if (m == ST_FUNCTIONAL) {
            if (nt < 7) return 203;
            if (!getDouble(tok[5], &coeff) || !getDouble(tok[6], &expon)) return 211;
            n = 7;
        } else {
            curve = curveOf(tok[5]);
            if (curve < 0) return 209;
            n = 6;
        }
        int flap = 0;
        if (nt > n) { flap = kfind(tok[n], kNoYes); if (flap < 0) return 205; }
        net.linkType[j] = OUTLET;
        net.offset1[j] = crest <= kMissing ? crest : crest / u;
        net.offset2[j] = net.offset1[j];
        net.ncC1[j] = coeff;
        net.ncC2[j] = expon;
        net.ncCurve[j] = curve;
        net.hasFlapGate[j] = flap > 0;
        net.ncSub[j] = ctype;
        double zero[4] = {0, 0, 0, 0};
        setXsectParams(net.xsect[j], X_DUMMY, zero, u);
        return 0;
    }
    }
    return 0;
}

// xsect_setParams (xsect.c:216-634)
bool setXsectParams(Xsect& x, int type, double p[4], double ucf)
{
    const double* ct = &SWX_CIRC_TABLES[0][0];
    if (type != X_DUMMY && p[0] <= 0.0) return false;
    x.type = type;
    auto g = [&]() { return geomOf(x); };
    switch (type) {
    case X_DUMMY:
        x.yFull = x.wMax = x.aFull = x.rFull = x.sFull = x.sMax = 1.E-6;
        break;
    case X_CIRCULAR:
        x.yFull = p[0] / ucf;
        x.wMax = x.yFull;
        x.aFull = kPi / 4.0 * x.yFull * x.yFull;
        x.rFull = 0.2500 * x.yFull;
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        x.sMax = 1.08 * x.sFull;
        x.ywMax = 0.5 * x.yFull;
        break;
    case X_FORCE_MAIN:
        x.yFull = p[0] / ucf;
        x.wMax = x.yFull;
        x.aFull = kPi / 4.0 * x.yFull * x.yFull;
        x.rFull = 0.2500 * x.yFull;
        x.sFull = x.aFull * pow(x.rFull, 0.63);
        x.sMax = 1.06949 * x.sFull;
        x.ywMax = 0.5 * x.yFull;
        x.rBot = p[1];                        // C-factor or roughness height
        break;
    case X_FILLED_CIRCULAR: {
        if (p[1] >= p[0]) return false;
        x.yFull = p[0] / ucf;
        x.wMax = x.yFull;
        x.aFull = kPi / 4.0 * x.yFull * x.yFull;
        x.rFull = 0.2500 * x.yFull;
        x.yBot = p[1] / ucf;
        x.aBot = x.aFull * lookup(x.yBot / x.yFull, SWX_TA(ct), SWX_CIRC_N);
        x.sBot = getWofY(g(), x.yBot, ct);    // the filled-circle W(y), yFull still whole
        x.rBot = x.aBot / (x.rFull * lookup(x.yBot / x.yFull, SWX_TR(ct), SWX_CIRC_N));
        x.aFull -= x.aBot;
        x.rFull = x.aFull / (kPi * x.yFull - x.rBot + x.sBot);
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        x.sMax = 1.08 * x.sFull;
        x.yFull -= x.yBot;
        x.ywMax = 0.5 * x.yFull;
        break;
    }
    case X_EGGSHAPED: case X_HORSESHOE: case X_GOTHIC: case X_CATENARY: case X_SEMIELLIPTICAL:
    case X_BASKETHANDLE: case X_SEMICIRCULAR: {
        // per shape: aFull/y^2, rFull/y, sMax/sFull, wMax/y, ywMax/y (xsect.c:295-363)
        static const double k[7][5] = {
            {0.5105, 0.1931, 1.065, 2. / 3., 0.64},       // EGGSHAPED
            {0.8293, 0.2538, 1.077, 1.0, 0.5},            // HORSESHOE
            {0.6554, 0.2269, 1.065, 0.84, 0.45},          // GOTHIC
            {0.70277, 0.23172, 1.05, 0.9, 0.25},          // CATENARY
            {0.785, 0.242, 1.045, 1.0, 0.15},             // SEMIELLIPTICAL
            {0.7862, 0.2464, 1.06078, 0.944, 0.2},        // BASKETHANDLE
            {1.2697, 0.2946, 1.06637, 1.64, 0.15}};       // SEMICIRCULAR
        int i = (type == X_EGGSHAPED) ? 0 : (type == X_HORSESHOE) ? 1 : type - X_GOTHIC + 2;
        x.yFull = p[0] / ucf;
        x.aFull = k[i][0] * x.yFull * x.yFull;
        x.rFull = k[i][1] * x.yFull;
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        x.sMax = k[i][2] * x.sFull;
        x.wMax = (i == 0 ? 2. / 3. : k[i][3]) * x.yFull;
        x.ywMax = k[i][4] * x.yFull;
        break;
    }
    case X_RECT_CLOSED: {
        if (p[1] <= 0.0) return false;
        x.yFull = p[0] / ucf;
        x.wMax = p[1] / ucf;
        x.aFull = x.yFull * x.wMax;
        x.rFull = x.aFull / (2.0 * (x.yFull + x.wMax));
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        double aMax = 0.97 * x.aFull;
        x.sMax = aMax * pow(rectClosedRofA(g(), aMax), 2. / 3.);
        x.ywMax = x.yFull;
        break;
    }
    case X_RECT_OPEN:
        if (p[1] <= 0.0) return false;
        x.yFull = p[0] / ucf;
        x.wMax = p[1] / ucf;
        if (p[2] < 0.0 || p[2] > 2.0) return false;
        x.sBot = p[2];
        x.aFull = x.yFull * x.wMax;
        x.rFull = x.aFull / ((2.0 - x.sBot) * x.yFull + x.wMax);
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        x.sMax = x.sFull;
        x.ywMax = x.yFull;
        break;
    case X_RECT_TRIANG: {
        if (p[1] <= 0.0 || p[2] <= 0.0) return false;
        x.yFull = p[0] / ucf;
        x.wMax = p[1] / ucf;
        x.yBot = p[2] / ucf;
        x.ywMax = x.yFull;
        x.aBot = x.yBot * x.wMax / 2.0;
        x.sBot = x.wMax / x.yBot / 2.0;
        x.rBot = sqrt(1. + x.sBot * x.sBot);
        x.aFull = x.wMax * (x.yFull - x.yBot / 2.0);
        x.rFull = x.aFull / (2.0 * x.yBot * x.rBot + 2.0 * (x.yFull - x.yBot) + x.wMax);
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        double aMax = SWX_RECT_TRIANG_ALFMAX * x.aFull;
        x.sMax = aMax * pow(rectTriangRofA(g(), aMax), 2. / 3.);
        break;
    }
    case X_RECT_ROUND: {
        if (p[1] <= 0.0) return false;
        if (p[2] < p[1] / 2.0) p[2] = p[1] / 2.0;
        x.yFull = p[0] / ucf;
        x.wMax = p[1] / ucf;
        x.rBot = p[2] / ucf;
        double theta = 2.0 * asin(x.wMax / 2.0 / x.rBot);
        x.aBot = x.rBot * x.rBot / 2.0 * (theta - sin(theta));
        x.sBot = kPi * x.rBot * x.rBot * pow(x.rBot / 2.0, 2. / 3.);
        x.yBot = x.rBot * (1.0 - cos(theta / 2.0));
        if (x.yBot > x.yFull) return false;
        x.ywMax = x.yFull;
        x.aFull = x.wMax * (x.yFull - x.yBot) + x.aBot;
        x.rFull = x.aFull / (x.rBot * theta + 2.0 * (x.yFull - x.yBot) + x.wMax);
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        double aMax = SWX_RECT_ROUND_ALFMAX * x.aFull;
        x.sMax = aMax * pow(rectRoundRofA(g(), aMax, ct), 2. / 3.);
        break;
    }
    case X_MOD_BASKET: {
        if (p[1] <= 0.0) return false;
        if (p[2] < p[1] / 2.0) p[2] = p[1] / 2.0;
        x.yFull = p[0] / ucf;
        x.wMax = p[1] / ucf;
        x.rBot = p[2] / ucf;
        double theta = 2.0 * asin(x.wMax / 2.0 / x.rBot);
        x.sBot = theta;
        x.yBot = x.rBot * (1.0 - cos(theta / 2.0));
        if (x.yBot > x.yFull) return false;
        x.ywMax = x.yFull - x.yBot;
        x.aBot = x.rBot * x.rBot / 2.0 * (theta - sin(theta));
        x.aFull = (x.yFull - x.yBot) * x.wMax + x.aBot;
        x.rFull = x.aFull / (x.rBot * theta + 2.0 * (x.yFull - x.yBot) + x.wMax);
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        x.sMax = getSofA(g(), amaxRatio(X_MOD_BASKET) * x.aFull, ct);
        break;
    }
    case X_TRAPEZOIDAL:
        if (p[1] < 0.0 || p[2] < 0.0 || p[3] < 0.0) return false;
        x.yFull = p[0] / ucf;
        x.ywMax = x.yFull;
        x.yBot = p[1] / ucf;
        x.sBot = (p[2] + p[3]) / 2.0;
        if (x.yBot == 0.0 && x.sBot == 0.0) return false;
        x.rBot = sqrt(1.0 + p[2] * p[2]) + sqrt(1.0 + p[3] * p[3]);
        x.wMax = x.yBot + x.yFull * (p[2] + p[3]);
        x.aFull = (x.yBot + x.sBot * x.yFull) * x.yFull;
        x.rFull = x.aFull / (x.yBot + x.yFull * x.rBot);
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        x.sMax = x.sFull;
        break;
    case X_TRIANGULAR:
        if (p[1] <= 0.0) return false;
        x.yFull = p[0] / ucf;
        x.wMax = p[1] / ucf;
        x.ywMax = x.yFull;
        x.sBot = x.wMax / x.yFull / 2.;
        x.rBot = sqrt(1. + x.sBot * x.sBot);
        x.aFull = x.yFull * x.yFull * x.sBot;
        x.rFull = x.aFull / (2.0 * x.yFull * x.rBot);
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        x.sMax = x.sFull;
        break;
    case X_PARABOLIC:
        if (p[1] <= 0.0) return false;
        x.yFull = p[0] / ucf;
        x.wMax = p[1] / ucf;
        x.ywMax = x.yFull;
        x.rBot = x.wMax / 2.0 / sqrt(x.yFull);
        x.aFull = (2. / 3.) * x.yFull * x.wMax;
        x.rFull = getRofY(g(), x.yFull, ct);
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        x.sMax = x.sFull;
        break;
    case X_POWERFUNC:
        if (p[1] <= 0.0 || p[2] <= 0.0) return false;
        x.yFull = p[0] / ucf;
        x.wMax = p[1] / ucf;
        x.ywMax = x.yFull;
        x.sBot = 1.0 / p[2];
        x.rBot = x.wMax / (x.sBot + 1) / pow(x.yFull, x.sBot);
        x.aFull = x.yFull * x.wMax / (x.sBot + 1);
        x.rFull = getRofY(g(), x.yFull, ct);
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        x.sMax = x.sFull;
        break;
    case X_HORIZ_ELLIPSE:
    case X_VERT_ELLIPSE: {
        bool horiz = type == X_HORIZ_ELLIPSE;
        if (p[1] == 0.0) p[2] = p[0];
        if (p[2] > 0.0) {                        // standard size code
            int i = (int)floor(p[2]) - 1;
            if (i < 0 || i >= SWX_N_ELLIPSE_MINOR) return false;
            double minor = SWX_ELLIPSE_MINOR[i] / 12., major = SWX_ELLIPSE_MAJOR[i] / 12.;
            x.yFull = horiz ? minor : major;
            x.wMax = horiz ? major : minor;
            x.aFull = SWX_ELLIPSE_AFULL[i];
            x.rFull = SWX_ELLIPSE_RFULL[i];
        } else if (horiz) {
            x.yFull = p[0] / ucf;
            if (p[1] < 0.0) return false;
            x.wMax = p[1] / ucf;
            x.aFull = 1.2692 * x.yFull * x.yFull;
            x.rFull = 0.3061 * x.yFull;
        } else {
            if (p[1] < 0.0) return false;
            x.yFull = p[0] / ucf;
            x.wMax = p[1] / ucf;
            x.aFull = 1.2692 * x.wMax * x.wMax;
            x.rFull = 0.3061 * x.wMax;
        }
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        x.sMax = x.sFull;
        x.ywMax = 0.48 * x.yFull;
        break;
    }
    case X_ARCH:
        if (p[1] == 0.0) p[2] = p[0];
        if (p[2] > 0.0) {
            int i = (int)floor(p[2]) - 1;
            if (i < 0 || i >= SWX_N_ARCH_YFULL) return false;
            x.yFull = SWX_ARCH_YFULL[i] / 12.;
            x.wMax = SWX_ARCH_WMAX[i] / 12.;
            x.aFull = SWX_ARCH_AFULL[i];
            x.rFull = SWX_ARCH_RFULL[i];
        } else {
            if (p[1] < 0.0) return false;
            x.yFull = p[0] / ucf;
            x.wMax = p[1] / ucf;
            x.aFull = 0.7879 * x.yFull * x.wMax;
            x.rFull = 0.2991 * x.yFull;
        }
        x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
        x.sMax = x.sFull;
        x.ywMax = 0.28 * x.yFull;
        break;
    case X_CUSTOM:                  // parameters come from its shape curve (conduit_validate)
        break;
    default:
        return false;
    }
    return true;
}

int Project::readXsect(std::vector<char*>& tok)  // link.c:162-267
{
    int nt = (int)tok.size();
    if (nt < 3) return 203;
    auto it = net.linkIndex.find(tok[0]);
    if (it == net.linkIndex.end()) return 209;
    int j = it->second;
    int k = kfind(tok[1], kXsectWords);
    if (k < 0) return 205;
    if (net.linkType[j] == CONDUIT) net.barrels[j] = 1;
    net.xsect[j].culvertCode = 0;
    if (k == X_STREET) {                               // link.c:205-213
        auto t = net.streetIndex.find(tok[2]);
        if (t == net.streetIndex.end()) return 209;
        net.xsect[j].type = k;
        net.xsect[j].transect = t->second;
        return 0;
    }
    if (k == X_IRREGULAR) {                            // link.c:196-203
        auto t = net.transectIndex.find(tok[2]);
        if (t == net.transectIndex.end()) return 209;
        net.xsect[j].type = k;
        net.xsect[j].transect = t->second;
        return 0;
    }
    if (nt < 6) return 203;
    double x[4] = {0, 0, 0, 0};
    if (k == X_CUSTOM) {                               // link.c:221-230
        if (!getDouble(tok[2], &x[0]) || x[0] <= 0.0) return 211;
        auto c = net.curveIndex.find(tok[3]);
        if (c == net.curveIndex.end()) return 209;
        net.xsect[j].type = k;
        net.xsect[j].transect = c->second;
        net.xsect[j].yFull = x[0] / ucfLength();
    } else
    for (int i = 2; i <= 5; i++)
        if (!getDouble(tok[i], &x[i - 2])) return 211;
    if (net.linkType[j] != CONDUIT && k == X_RECT_OPEN) { x[2] = 0.0; x[3] = 0.0; }
    if (!setXsectParams(net.xsect[j], k, x, ucfLength())) return 211;
    if (net.linkType[j] != CONDUIT) return 0;
    if (nt >= 7) {
        int i = atoi(tok[6]);
        if (i <= 0) return 211;
        net.barrels[j] = (int)(signed char)i;
    }
    if (nt >= 8) {
        int i = atoi(tok[7]);
        if (i < 0) return 211;
        net.xsect[j].culvertCode = i;
    }
    return 0;
}

int Project::readLoss(std::vector<char*>& tok)  // link.c:271-311
{
    int nt = (int)tok.size();
    if (nt < 4) return 203;
    auto it = net.linkIndex.find(tok[0]);
    if (it == net.linkIndex.end()) return 209;
    int j = it->second;
    double x[3], seep = 0.0;
    for (int i = 1; i <= 3; i++)
        if (!getDouble(tok[i], &x[i - 1]) || x[i - 1] < 0.0) return 211;
    int k = 0;
    if (nt >= 5) {
        k = kfind(tok[4], kNoYes);
        if (k < 0) return 205;
    }
    if (nt >= 6 && !getDouble(tok[5], &seep)) return 211;
    net.cLossInlet[j] = x[0];
    net.cLossOutlet[j] = x[1];
    net.cLossAvg[j] = x[2];
    net.hasFlapGate[j] = k;
    net.seepRate[j] = seep / ucfRainfall();
    return 0;
}

int Project::readPollutant(std::vector<char*>& tok)  // landuse.c:readPollutParams
{
    int nt = (int)tok.size();
    if (nt < 6) return 203;
    int j = net.pollutIndex.at(tok[0]);
    int k = kfind(tok[1], kQualUnitWords);
    if (k < 0) return 205;
    double x[4];
    for (int i = 2; i <= 4; i++)
        if (!getDouble(tok[i], &x[i - 2]) || x[i - 2] < 0.0) return 211;
    if (!getDouble(tok[5], &x[3])) return 211;
    double cDWF = 0.0, cInit = 0.0;
    if (nt >= 7 && kfind(tok[6], kNoYes) < 0) return 205;
    // co-pollutant (landuse.c:144-154): validated like the reference; it only
    // adds to runoff washoff (landuse_getCoPollutLoad), and a network without
    // subcatchments has none, so it leaves routing unchanged
    if (nt >= 9 && strcmp(tok[7], "*") != 0) {
        if (!net.pollutIndex.count(tok[7])) return 209;
        double coFrac;
        if (!getDouble(tok[8], &coFrac) || coFrac < 0.0) return 211;
    }
    if (nt >= 10 && (!getDouble(tok[9], &cDWF) || cDWF < 0.0)) return 211;
    if (nt >= 11 && (!getDouble(tok[10], &cInit) || cInit < 0.0)) return 211;
    Pollutant& p = net.pollut[j];
    p.units = k;
    double ucfMass = opt.unitSystem ? 1.0e-6 : 2.203e-6;
    p.mcf = (k == CU_MG) ? ucfMass : (k == CU_UG ? ucfMass / 1000.0 : 1.0);
    p.cRain = x[0];
    p.cGW = x[1];
    p.cRDII = x[2];
    p.kDecay = x[3] / kSecPerDay;
    p.cDWF = cDWF;
    p.cInit = cInit;
    return 0;
}

int Project::readInflow(std::vector<char*>& tok)  // inflow.c:41-134
{
    int nt = (int)tok.size();
    if (nt < 3) return 203;
    auto nit = net.nodeIndex.find(tok[0]);
    if (nit == net.nodeIndex.end()) return 209;
    ExtInflow in;
    in.node = nit->second;
    in.type = EXT_CONCEN;
    auto pit = net.pollutIndex.find(tok[1]);
    if (pit == net.pollutIndex.end()) {
        if (kmatch(tok[1], "FLOW")) in.param = -1;
        else return 209;
    } else {
        in.param = pit->second;
    }
    if (strlen(tok[2]) > 0) {
        auto t = net.tseriesIndex.find(tok[2]);
        if (t == net.tseriesIndex.end()) return 209;
        in.tseries = t->second;
    }
    double cf = 1.0, sf = 1.0, baseline = 0.0;
    if (in.param == -1) {
        in.type = EXT_FLOW;
        cf = 1.0 / ucfFlow();
    }
    if (nt >= 4 && in.param > -1) {
        if (kmatch(tok[3], "CONCEN")) in.type = EXT_CONCEN;
        else if (kmatch(tok[3], "MASS")) in.type = EXT_MASS;
        else return 205;
        if (nt >= 5 && in.type == EXT_MASS) {
            if (!getDouble(tok[4], &cf)) return 211;
            if (cf <= 0.0) return 211;
        }
    }
    if (nt >= 6 && !getDouble(tok[5], &sf)) return 211;
    if (nt >= 7 && !getDouble(tok[6], &baseline)) return 211;
    if (nt >= 8) {
        auto p = net.patternIndex.find(tok[7]);
        if (p == net.patternIndex.end()) return 209;
        in.basePat = p->second;
    }
    if (in.type == EXT_MASS) cf /= kLperFT3;
    in.cFactor = cf;
    in.sFactor = sf;
    in.baseline = baseline;
    // replace an existing inflow for the same constituent (inflow.c:153-184)
    long long key = (long long)in.node * 1024 + (in.param + 1);
    auto it = extKey_.find(key);
    if (it != extKey_.end()) { net.extInflows[it->second] = in; return 0; }
    extKey_.emplace(key, (int)net.extInflows.size());
    net.extInflows.push_back(in);
    return 0;
}

int Project::readDwf(std::vector<char*>& tok)  // inflow.c:237-306
{
    int nt = (int)tok.size();
    if (nt < 3) return 203;
    auto nit = net.nodeIndex.find(tok[0]);
    if (nit == net.nodeIndex.end()) return 209;
    DwfInflow in;
    in.node = nit->second;
    auto pit = net.pollutIndex.find(tok[1]);
    if (pit == net.pollutIndex.end()) {
        if (kmatch(tok[1], "FLOW")) in.param = -1;
        else return 209;
    } else {
        in.param = pit->second;
    }
    double x;
    if (!getDouble(tok[2], &x)) return 211;
    if (in.param == -1) x /= ucfFlow();
    in.avgValue = x;
    for (int i = 3; i < 7 && i < nt; i++) {
        if (strlen(tok[i]) == 0) continue;
        auto p = net.patternIndex.find(tok[i]);
        if (p == net.patternIndex.end()) return 209;
        in.patterns[i - 3] = p->second;
    }
    long long key = (long long)in.node * 1024 + (in.param + 1);
    auto it = dwfKey_.find(key);
    if (it != dwfKey_.end()) { net.dwfInflows[it->second] = in; return 0; }
    dwfKey_.emplace(key, (int)net.dwfInflows.size());
    net.dwfInflows.push_back(in);
    return 0;
}

int Project::readPattern(std::vector<char*>& tok)  // inflow.c:410-452
{
    int nt = (int)tok.size();
    if (nt < 2) return 203;
    Pattern& p = net.patterns[net.patternIndex.at(tok[0])];
    int n = 1;
    if (p.type < 0) {
        int k = kfind(tok[1], kPatternWords);
        if (k < 0) return 205;
        p.type = k;
        n = 2;
    }
    while (nt > n && p.count < 24) {
        if (!getDouble(tok[n], &p.factor[p.count])) return 211;
        p.count++;
        n++;
    }
    return 0;
}

int Project::readTimeseries(std::vector<char*>& tok)  // table.c:113-202
{
    int nt = (int)tok.size();
    if (nt < 3) return 203;
    Tseries& ts = net.tseries[net.tseriesIndex.at(tok[0])];
    if (kmatch(tok[1], "FILE")) {                       // table.c:143-149
        std::string fname = tok[2];
        bool rel = !(strchr(fname.c_str(), ':') || fname[0] == '\\' || fname[0] == '/');
        ts.file = rel ? inpDir + fname : fname;
        return 0;
    }
    double x = 0.0, y, d, t;
    int k = 1, state = 1;
    while (k < nt) {
        switch (state) {
        case 1:
            if (strToDate(tok[k], &d)) {
                ts.lastDate = d;
                k++;
            }
            state = 2;
            break;
        case 2:
            if (k >= nt) return 203;
            if (getDouble(tok[k], &t)) t /= 24.0;
            else if (!strToTime(tok[k], &t)) return 211;
            x = ts.lastDate + t;
            k++;
            state = 3;
            break;
        case 3:
            if (k >= nt) return 203;
            if (!getDouble(tok[k], &y)) return 211;
            ts.x.push_back(x);
            ts.y.push_back(y);
            k++;
            state = 1;
            break;
        }
    }
    return 0;
}

// [FILES] USE|SAVE FileType FileName (iface.c:66-134).  Hot start files are
// supported; rainfall / runoff files belong to the runoff model (no
// subcatchments here) and are ignored; routing interface files change the
// routed inflows and are rejected.
int Project::readFiles(std::vector<char*>& tok)
{
    static const char* const kModes[] = {"NO", "SCRATCH", "USE", "SAVE", nullptr};
    static const char* const kTypes[] = {"RAINFALL", "RUNOFF", "HOTSTART", "RDII", "INFLOWS",
                                         "OUTFLOWS", nullptr};
    int nt = (int)tok.size();
    if (nt < 2) return 203;
    int k = kfind(tok[0], kModes);
    if (k < 0) return 205;
    int j = kfind(tok[1], kTypes);
    if (j < 0) return 205;
    if (nt < 3) return 0;
    std::string fname = tok[2];
    // addAbsolutePath (swmm5.c:1620-1633)
    bool rel = !(strchr(fname.c_str(), ':') || fname[0] == '\\' || fname[0] == '/');
    if (rel) fname = inpDir + fname;
    switch (j) {
    case 2:
        if (k == 2) hotstartUse = fname;
        else if (k == 3) hotstartSave = fname;
        return 0;
    case 4:
        if (k != 2) return 203;
        break;
    case 5:
        if (k != 3) return 203;
        break;
    case 3:
        if (k != 2 && k != 3) return 0;
        break;
    default:
        return 0;
    }
    return setError(200, std::string("ERROR 200: ") + kTypes[j] +
                             " interface files are not supported by the MI355X dynamic-wave engine");
}

// openHotstartFile1 + readRouting (hotstart.c:95-171, 252-330): versions 1-4.
// The file must describe the same object counts and flow units; node depth,
// lateral inflow and quality, and link flow, depth and setting are read as
// float32.
int Project::readHotstart()
{
    FILE* f = fopen(hotstartUse.c_str(), "rb");
    if (!f) return setError(331, "ERROR 331: cannot open hot start interface file " + hotstartUse + ".");
    auto fmt = [&]() {
        fclose(f);
        return setError(333, "ERROR 333: incompatible data found in hot start interface file.");
    };
    char stamp[16] = {0};
    int version = 0;
    if (fread(stamp, 1, 15, f) == 15) {
        if (!strcmp(stamp, "SWMM5-HOTSTART4")) version = 4;
        else if (!strcmp(stamp, "SWMM5-HOTSTART3")) version = 3;
        else if (!strcmp(stamp, "SWMM5-HOTSTART2")) version = 2;
    }
    if (!version) {
        rewind(f);
        char s1[15] = {0};
        if (fread(s1, 1, 14, f) != 14 || strcmp(s1, "SWMM5-HOTSTART")) return fmt();
        version = 1;
    }
    int nSub = 0, nLand = 0, nNode = -1, nLink = -1, nPoll = -1, units = -1;
    auto rdi = [&](int* x) { return fread(x, sizeof(int), 1, f) == 1; };
    if (version >= 2 && !rdi(&nSub)) return fmt();
    if (version >= 3 && !rdi(&nLand)) return fmt();
    if (!rdi(&nNode) || !rdi(&nLink) || !rdi(&nPoll) || !rdi(&units)) return fmt();
    int nn = net.nNodes(), nl = net.nLinks(), P = net.nPollut();
    if (nSub != 0 || nLand != 0 || nNode != nn || nLink != nl || nPoll != P || units != opt.flowUnits)
        return fmt();
    // readRunoff (version >= 3) has nothing to read without subcatchments;
    // version 2's groundwater records likewise
    auto rdf = [&](double* y) {
        float x;
        if (fread(&x, sizeof(float), 1, f) != 1 || x != x) {
            setError(335, "ERROR 335: error in reading from hot start interface file.");
            return false;
        }
        *y = x;
        return true;
    };
    State& s = st;
    double x;
    for (int i = 0; i < nn; i++) {
        if (!rdf(&s.newDepth[i]) || !rdf(&s.newLatFlow[i])) break;
        if (version >= 4 && net.nodeType[i] == STORAGE && !rdf(&s.hrt[i])) break;
        bool ok = true;
        for (int p = 0; p < P && ok; p++) ok = rdf(&s.nNewQual[(size_t)p * nn + i]);
        for (int p = 0; version <= 2 && p < P && ok; p++) ok = rdf(&x);
        if (!ok) break;
    }
    for (int i = 0; i < nl && !errorCode; i++) {
        if (!rdf(&s.lNewFlow[i]) || !rdf(&s.lNewDepth[i]) || !rdf(&s.setting[i])) break;
        // link_setTargetSetting / link_setSetting: no effect on conduits
        bool ok = true;
        for (int p = 0; p < P && ok; p++) ok = rdf(&s.lNewQual[(size_t)p * nl + i]);
        if (!ok) break;
    }
    fclose(f);
    return errorCode;
}

int Project::saveHotstart()   // openHotstartFile2 + saveRouting (hotstart.c:175-250)
{
    if (hotstartSave.empty()) return 0;
    FILE* f = fopen(hotstartSave.c_str(), "w+b");
    if (!f) return setError(331, "ERROR 331: cannot open hot start interface file " + hotstartSave + ".");
    int nn = net.nNodes(), nl = net.nLinks(), P = net.nPollut();
    int hdr[6] = {0, 0, nn, nl, P, opt.flowUnits};
    fwrite("SWMM5-HOTSTART4", 1, 15, f);
    fwrite(hdr, sizeof(int), 6, f);
    std::vector<float> buf;
    buf.reserve((size_t)(nn + nl) * (3 + P));
    const State& s = st;
    for (int i = 0; i < nn; i++) {
        buf.push_back((float)s.newDepth[i]);
        buf.push_back((float)s.newLatFlow[i]);
        if (net.nodeType[i] == STORAGE) buf.push_back((float)s.hrt[i]);
        for (int p = 0; p < P; p++) buf.push_back((float)s.nNewQual[(size_t)p * nn + i]);
    }
    for (int i = 0; i < nl; i++) {
        buf.push_back((float)s.lNewFlow[i]);
        buf.push_back((float)s.lNewDepth[i]);
        buf.push_back((float)s.setting[i]);
        for (int p = 0; p < P; p++) buf.push_back((float)s.lNewQual[(size_t)p * nl + i]);
    }
    fwrite(buf.data(), sizeof(float), buf.size(), f);
    bool bad = ferror(f) != 0;
    fclose(f);
    if (bad) return setError(331, "ERROR 331: cannot open hot start interface file " + hotstartSave + ".");
    return 0;
}

int Project::readReport(std::vector<char*>& tok)  // report.c:report_readOptions
{
    int nt = (int)tok.size();
    if (nt < 2) return 203;
    static const char* const kReportWords[] = {"DISABLED", "INPUT", "SUBCATCH", "NODE", "LINK",
                                               "CONTINUITY", "FLOWSTATS", "CONTROL", "AVERAGES",
                                               "NODESTATS", nullptr};
    int k = kfind(tok[0], kReportWords);
    if (k < 0) return 205;
    if (k < 2 || k > 4) {
        int m = kfind(tok[1], kNoYes);
        if (m < 0) return 205;
        switch (k) {
        case 0: rpt.disabled = m; break;
        case 1: rpt.input = m; break;
        case 5: rpt.continuity = m; break;
        case 6: rpt.flowStats = m; break;
        case 7: rpt.controls = m; break;
        case 8: rpt.averages = m; break;
        default: break;
        }
        return 0;
    }
    int flag;
    if (strcasecmp(tok[1], "NONE") == 0) flag = 0;
    else if (strcasecmp(tok[1], "ALL") == 0) flag = 1;
    else {
        flag = 2;
        for (int t = 1; t < nt; t++) {
            if (k == 3) {
                auto it = net.nodeIndex.find(tok[t]);
                if (it == net.nodeIndex.end()) return 209;
                net.rptFlag[it->second] = 1;
            } else if (k == 4) {
                auto it = net.linkIndex.find(tok[t]);
                if (it == net.linkIndex.end()) return 209;
                net.linkRpt[it->second] = 1;
            }
        }
    }
    if (k == 2) rpt.subcatchAll = flag;
    else if (k == 3) rpt.nodesAll = flag;
    else rpt.linksAll = flag;
    return 0;
}

// ============================================================== validation
// link.c:1258-1300
static double conduitSlope(const Network& n, int j, const Options& o, int* warn)
{
    double length = n.lengthT[j];               // conduit_getLength
    double elev1 = n.offset1[j] + n.invertElev[n.node1[j]];
    double elev2 = n.offset2[j] + n.invertElev[n.node2[j]];
    double delta = fabs(elev1 - elev2), slope;
    if (delta < kMinDeltaZ) { (*warn)++; delta = kMinDeltaZ; }
    if (delta >= length) { (*warn)++; slope = delta / length; }
    else slope = delta / sqrt((length * length) - (delta * delta));
    if (o.minSlope > 0.0 && slope < o.minSlope) { (*warn)++; slope = o.minSlope; }
    if (elev1 < elev2) slope = -slope;
    return slope;
}

void Project::validateConduit(int j)  // link.c:992-1154 (supported shapes)
{
    Xsect& xs = net.xsect[j];
    if (xs.type < 0) { setError(117, "ERROR 117: no cross section defined for link " + net.linkId[j]); return; }
    if (xs.type == X_DUMMY && net.nodeType[net.node1[j]] == STORAGE) {   // link.c:1003-1011 (DW)
        setError(134, "ERROR 134: Node " + net.nodeId[net.node1[j]] + " has illegal DUMMY link connections.");
        return;
    }
    const XTable* tt = nullptr;
    if (xs.type == X_CUSTOM) {                         // xsect_setCustomXsectParams xsect.c:664-696
        int sh = (xs.transect >= 0 && xs.transect < (int)net.curveShape.size()) ? net.curveShape[xs.transect] : -1;
        if (sh < 0) { setError(119, "ERROR 119: invalid cross section for link " + net.linkId[j]); return; }
        const XTable& t = net.shapes[sh];
        double yFull = xs.yFull;
        xs.wMax = t.wMax * yFull;
        xs.aFull = t.aFull * yFull * yFull;
        xs.rFull = t.rFull * yFull;
        xs.sFull = xs.aFull * pow(xs.rFull, 2. / 3.);
        xs.sMax = t.sMax * yFull * yFull * pow(yFull, 2. / 3.);
        xs.aBot = t.aMax * yFull * yFull;
        tt = &t;
    } else if (xs.type == X_IRREGULAR || xs.type == X_STREET) {   // getTransectParams xsect.c:1323-1355
        const XTable& t = (xs.type == X_IRREGULAR) ? net.transects[xs.transect] : net.streets[xs.transect];
        xs.yFull = t.yFull;
        xs.wMax = t.wMax;
        xs.aFull = t.aFull;
        xs.rFull = t.rFull;
        xs.sFull = xs.aFull * pow(xs.rFull, 2. / 3.);
        xs.sMax = t.sMax;
        xs.aBot = t.aMax;
        net.roughness[j] = t.roughness;               // transect / street roughness (link.c:1018-1029)
        tt = &t;
    }
    if (tt) {
        // search the width table up to where the width decreases; depth of
        // the lowest widest point (xsect.c:684-695, 1343-1354)
        int iMax = 0;
        double wMax = tt->width.empty() ? 0.0 : tt->width[0];
        for (int i = 1; i < tt->nTbl; i++) {
            if (tt->width[i] < wMax) break;
            wMax = tt->width[i];
            iMax = i;
        }
        if (xs.type == X_CUSTOM) xs.ywMax = xs.yFull * (double)iMax / (double)(51 - 1);
        else xs.ywMax = xs.yFull * (double)iMax / ((double)(tt->nTbl) - 1);
        xs.tabOff = tt->blockOff;
    }
    // conduit_getLength (link.c:1195-1206): irregular channels use the flood
    // plain's length
    net.lengthT[j] = net.length[j];
    if (xs.type == X_IRREGULAR) net.lengthT[j] = net.length[j] / net.transects[xs.transect].lengthFactor;
    if (net.length[j] <= 0.0) { setError(111, "ERROR 111: invalid length for Conduit " + net.linkId[j]); return; }
    if (net.roughness[j] <= 0.0) { setError(113, "ERROR 113: invalid roughness for Conduit " + net.linkId[j]); return; }
    if (net.barrels[j] <= 0) { setError(114, "ERROR 114: invalid number of barrels for Conduit " + net.linkId[j]); return; }
    if (xs.type == X_FORCE_MAIN) {                     // link.c:1031-1037
        if (opt.forceMainEqn == FM_D_W) xs.rBot /= (opt.unitSystem ? 304.8 : 12.0);
        if (xs.rBot <= 0.0) { setError(119, "ERROR 119: invalid cross section for link " + net.linkId[j]); return; }
    }
    if (xs.aFull <= 0.0) { setError(119, "ERROR 119: invalid cross section for link " + net.linkId[j]); return; }
    if (net.offset1[j] < 0.0) { warnings++; net.offset1[j] = 0.0; }
    if (net.offset2[j] < 0.0) { warnings++; net.offset2[j] = 0.0; }
    if (xs.type == X_FILLED_CIRCULAR) {                // link.c:1069-1074
        net.offset1[j] += xs.yBot;
        net.offset2[j] += xs.yBot;
    }
    double slope = conduitSlope(net, j, opt, &warnings);
    net.slope[j] = slope;
    if (slope < 0.0 && xs.type != X_DUMMY) {           // conduit_reverse link.c:1158-1191
        std::swap(net.node1[j], net.node2[j]);
        std::swap(net.offset1[j], net.offset2[j]);
        std::swap(net.cLossInlet[j], net.cLossOutlet[j]);
        net.slope[j] = -net.slope[j];
        net.direction[j] *= -1;
        net.q0[j] = -net.q0[j];
    }
    double roughness = net.roughness[j];
    if (xs.type == X_IRREGULAR)                        // meandering channels (link.c:1097-1102)
        roughness *= sqrt(net.transects[xs.transect].lengthFactor);
    if (xs.type == X_FORCE_MAIN) {                     // forcemain_getEquivN forcmain.c:30-47
        double d = xs.yFull;
        if (opt.forceMainEqn == FM_H_W) roughness = 1.067 / xs.rBot * pow(d / net.slope[j], 0.04);
        else {
            double f = fmFricFactor(xs.rBot, d / 4.0, 1.0e12);
            roughness = sqrt(f / 185.0) * pow(d, (1. / 6.));
        }
    }
    double lengthFactor = 1.0;
    if (opt.lengtheningStep > 0.0 && xs.type != X_DUMMY) {   // link.c:1217-1254
        Geom g = geomOf(xs, net.xTab.data());
        double yFull = xs.yFull;
        if (isOpen(xs.type)) yFull = xs.aFull / getWofY(g, yFull, &SWX_CIRC_TABLES[0][0]);
        double vFull = kPhi / roughness * xs.sFull * sqrt(fabs(net.slope[j])) / xs.aFull;
        double tStep = (opt.lengtheningStep == 0.0) ? opt.routeStep
                                                    : gmin(opt.routeStep, opt.lengtheningStep);
        double ratio = (sqrt(kGravity * yFull) + vFull) * tStep / net.lengthT[j];
        lengthFactor = ratio > 1.0 ? ratio : 1.0;
    }
    if (lengthFactor != 1.0) {
        net.modLength[j] = lengthFactor * net.lengthT[j];
        slope /= lengthFactor;
        roughness = roughness / sqrt(lengthFactor);
    }
    if (xs.type == X_FORCE_MAIN) {                     // forcemain_getRoughFactor forcmain.c:51-70
        if (opt.forceMainEqn == FM_H_W) {
            double r = 1.318 * xs.rBot * pow(lengthFactor, 0.54);
            xs.sBot = kGravity / pow(r, 1.852);
        } else {
            xs.sBot = 1.0 / 8.0 / lengthFactor;
        }
    }
    net.roughFactor[j] = kGravity * ((roughness / kPhi) * (roughness / kPhi));
    net.beta[j] = (xs.type == X_DUMMY) ? 0.0 : kPhi * sqrt(fabs(slope)) / roughness;
    net.qFull[j] = xs.sFull * net.beta[j];
    net.qMax[j] = xs.sMax * net.beta[j];
    double aa = net.beta[j] / sqrt(32.2) * pow(xs.yFull, 0.1666667) * 0.3;
    net.superCritical[j] = (aa >= 1.0) ? 1 : 0;
    net.hasLosses[j] = (net.cLossInlet[j] == 0.0 && net.cLossOutlet[j] == 0.0 &&
                        net.cLossAvg[j] == 0.0) ? 0 : 1;
}

// pump_validate / orifice_validate / weir_validate (link.c:1473-1530,
// 1696-1725, 2102-2152) and the crest check of link_validate (link.c:421-438)
void Project::validateRegulator(int j)
{
    const double* ct = &SWX_CIRC_TABLES[0][0];
    Xsect& xs = net.xsect[j];
    int type = net.linkType[j];
    if (type == PUMP) {
        xs.yFull = 0.0;
        int m = net.ncCurve[j];
        if (m < 0) net.ncSub[j] = PT_IDEAL;
        else {
            const Curve& c = net.curves[m];
            if (c.type < CV_PUMP1 || c.type > CV_PUMP5) {
                setError(143, "ERROR 143: invalid pump curve for Pump " + net.linkId[j]);
                return;
            }
            net.ncSub[j] = c.type - CV_PUMP1;
            if (!c.x.empty()) {
                double q = c.y[0];
                net.ncXMin[j] = c.x[0];
                net.ncXMax[j] = c.x[0];
                for (size_t i = 1; i < c.x.size(); i++) {
                    q = gmax(c.y[i], q);
                    net.ncXMax[j] = c.x[i];
                }
                net.qFull[j] = q / ucfFlow();
            }
        }
        if (net.ncYOn[j] > 0.0 && net.ncYOn[j] <= net.ncYOff[j]) {
            setError(145, "ERROR 145: pump startup depth not higher than shutoff depth for Pump " + net.linkId[j]);
            return;
        }
        if (net.ncSub[j] == PT_TYPE1) {
            int n1 = net.node1[j];
            if (net.nodeType[n1] != STORAGE)
                net.fullVolume[n1] = gmax(net.fullVolume[n1], net.ncXMax[j] / ucfVolume());
        }
        return;
    }
    if (type == ORIFICE) {
        if (xs.type != X_RECT_CLOSED && xs.type != X_CIRCULAR) {
            setError(121, "ERROR 121: invalid cross section shape for regulator " + net.linkId[j]);
            return;
        }
        if (net.offset1[j] < 0.0) net.offset1[j] = 0.0;
        net.ncLength[j] = 2.0 * opt.routeStep * sqrt(kGravity * xs.yFull);
        net.ncLength[j] = gmax(200.0, net.ncLength[j]);
    } else if (type == WEIR) {
        int w = net.ncSub[j];
        bool ok = true;
        if (w == WR_TRANSVERSE || w == WR_SIDEFLOW || w == WR_ROADWAY) { ok = xs.type == X_RECT_OPEN; net.ncSlope[j] = 0.0; }
        else if (w == WR_VNOTCH) { ok = xs.type == X_TRIANGULAR; if (ok) net.ncSlope[j] = xs.sBot; }
        else if (w == WR_TRAPEZOIDAL) { ok = xs.type == X_TRAPEZOIDAL; if (ok) net.ncSlope[j] = xs.sBot; }
        if (!ok) {
            setError(121, "ERROR 121: invalid cross section shape for regulator " + net.linkId[j]);
            return;
        }
        if (net.offset1[j] < 0.0) net.offset1[j] = 0.0;
        net.ncLength[j] = 2.0 * opt.routeStep * sqrt(kGravity * xs.yFull);
        net.ncLength[j] = gmax(200.0, net.ncLength[j]);
    }
    // crest below the downstream invert (DW: raised, link.c:421-438)
    int n1 = net.node1[j], n2 = net.node2[j];
    if (net.invertElev[n1] + net.offset1[j] < net.invertElev[n2]) {
        net.offset1[j] = net.invertElev[n2] - net.invertElev[n1];
        warnings++;
    }
    (void)ct;
}

void Project::validate()  // project.c:186-270
{
    int nn = net.nNodes(), nl = net.nLinks();
    for (auto& ts : net.tseries) {
        // an external file's entries (table_validate / table_parseFileLine,
        // table.c:290-330, 833-895): "date time value" or "time value" lines,
        // the date carried from the last dated line; ';' starts a comment
        if (ts.file.empty()) continue;
        FILE* fp = fopen(ts.file.c_str(), "rt");
        if (!fp) { setError(361, "ERROR 361: could not open external file used for Time Series " + ts.id); return; }
        char line[1025];
        bool bad = false;
        while (fgets(line, sizeof line, fp)) {
            char s1[50] = "", s2[50] = "", s3[50] = "";
            int n = sscanf(line, "%49s %49s %49s", s1, s2, s3);
            if (n <= 0 || s1[0] == ';') continue;
            double d, t, y;
            const char *tStr, *yStr;
            if (n == 2) { d = ts.lastDate; tStr = s1; yStr = s2; }
            else if (n == 3) {
                if (!strToDate(s1, &d)) { bad = true; break; }
                ts.lastDate = d;
                tStr = s2;
                yStr = s3;
            } else { bad = true; break; }
            if (getDouble(tStr, &t)) t /= 24.0;
            else if (!strToTime(tStr, &t)) { bad = true; break; }
            if (!getDouble(yStr, &y)) { bad = true; break; }
            ts.x.push_back(d + t);
            ts.y.push_back(y);
        }
        fclose(fp);
        if (bad || ts.x.empty()) { setError(363, "ERROR 363: invalid data in external file used for Time Series " + ts.id); return; }
    }
    for (auto& ts : net.tseries)
        for (size_t i = 1; i < ts.x.size(); i++)
            if (ts.x[i] <= ts.x[i - 1]) { setError(173, "ERROR 173: time series " + ts.id + " has its data out of sequence."); return; }
    climateValidate();
    if (opt.evapType == 2) {
        // the reference walks the series' shared entry cursor for evaporation
        // (table_getNextEntry); a series another object also reads would
        // interleave two walks of that cursor, which is not modelled
        bool shared = false;
        for (const auto& in : net.extInflows) shared = shared || in.tseries == opt.evapSeries;
        for (int s : net.outfallSeries) shared = shared || s == opt.evapSeries;
        if (shared) {
            setError(200, "ERROR 200: an evaporation time series that also feeds an inflow or an outfall "
                          "is not supported by the MI355X engine");
            return;
        }
    }
    for (const Divider& dv : net.dividers) {              // divider_validate (node.c:1216-1247)
        int i = dv.link;
        if (i < 0 || (net.node1[i] != dv.node && net.node2[i] != dv.node)) {
            setError(136, "ERROR 136: invalid diverted link for flow divider node " + net.nodeId[dv.node]);
            return;
        }
        if (dv.type == 2) {
            if (dv.dhMax <= 0.0 || dv.cWeir <= 0.0) {
                setError(137, "ERROR 137: invalid parameters for weir divider node " + net.nodeId[dv.node]);
                return;
            }
            double qMax = dv.cWeir * pow(dv.dhMax, 1.5) / ucfFlow();
            if (dv.qMin > qMax) {
                setError(137, "ERROR 137: invalid parameters for weir divider node " + net.nodeId[dv.node]);
                return;
            }
        }
    }
    buildXTables();                                      // shape curves (project.c:220-231)
    if (errorCode) return;
    for (size_t t = 0; t < net.transects.size(); t++)
        if (!net.transects[t].valid) {
            // a transect never validated has no geometry (aFull = 0, link.c:1052)
            for (int j = 0; j < nl; j++)
                if (net.xsect[j].type == X_IRREGULAR && net.xsect[j].transect == (int)t) {
                    setError(119, "ERROR 119: invalid cross section for link " + net.linkId[j]);
                    return;
                }
        }
    for (int j = 0; j < nl; j++) {
        if (opt.linkOffsetsElev) {                       // link.c:468-504
            for (int e = 0; e < 2; e++) {
                double& off = e == 0 ? net.offset1[j] : net.offset2[j];
                double elev = net.invertElev[e == 0 ? net.node1[j] : net.node2[j]];
                if (off <= kMissing) { off = 0.0; continue; }
                off -= elev;
                if (off >= 0.0) continue;
                if (off >= -kMinDeltaZ) { off = 0.0; continue; }
                warnings++;
                off = 0.0;
            }
        }
        if (net.linkType[j] == CONDUIT) validateConduit(j);
        else validateRegulator(j);
        if (errorCode) return;
        // link.c:440-463: not for pumps and bottom orifices; storage units
        // without surcharge keep their depth; downstream end for conduits only
        if (net.linkType[j] == PUMP || (net.linkType[j] == ORIFICE && net.ncSub[j] == OR_BOTTOM)) continue;
        int n = net.node1[j];
        if (net.nodeType[n] != STORAGE || net.surDepth[n] > 0.0)
            net.fullDepth[n] = gmax(net.fullDepth[n], net.offset1[j] + net.xsect[j].yFull);
        n = net.node2[j];
        if ((net.nodeType[n] != STORAGE || net.surDepth[n] > 0.0) && net.linkType[j] == CONDUIT)
            net.fullDepth[n] = gmax(net.fullDepth[n], net.offset2[j] + net.xsect[j].yFull);
    }
    for (int j = 0; j < nn; j++) {
        if (net.initDepth[j] > net.fullDepth[j] + net.surDepth[j]) {
            setError(138, "ERROR 138: initial depth greater than maximum depth for Node " + net.nodeId[j]);
            return;
        }
        if (net.nodeType[j] == STORAGE) {                // node_validate (node.c:219-222)
            StorageGeom g = storageGeom(j);
            g.fullVolume = 0.0;
            if (storageVolume(g, net.fullDepth[j]) < 0.0) {
                setError(119, "ERROR 119: negative storage volume at full depth for Node " + net.nodeId[j]);
                return;
            }
        }
    }
    // DWF pattern ordering (inflow.c:331-354)
    for (auto& d : net.dwfInflows) {
        int tmp[4] = {-1, -1, -1, -1};
        for (int i = 0; i < 4; i++)
            if (d.patterns[i] >= 0) tmp[net.patterns[d.patterns[i]].type] = d.patterns[i];
        for (int i = 0; i < 4; i++) d.patterns[i] = tmp[i];
    }
    if (opt.routeStep > (double)opt.wetStep) { warnings++; opt.routeStep = opt.wetStep; }
    // report flags
    if (rpt.nodesAll == 1) for (int j = 0; j < nn; j++) net.rptFlag[j] = 1;
    if (rpt.linksAll == 1) for (int j = 0; j < nl; j++) net.linkRpt[j] = 1;
    // dynwave_validate (dynwave.c:177-191)
    if (opt.minRouteStep > opt.routeStep) opt.minRouteStep = opt.routeStep;
    if (opt.minRouteStep < 0.001) opt.minRouteStep = 0.001;
    if (opt.minSurfArea == 0.0) opt.minSurfArea = 12.566;
    else opt.minSurfArea /= ucfLength() * ucfLength();
    if (opt.headTol == 0.0) opt.headTol = 0.005;
    else opt.headTol /= ucfLength();
    if (opt.maxTrials == 0) opt.maxTrials = 8;
    // toposort DW degree (toposort.c:57-90)
    for (int j = 0; j < nn; j++) net.degree[j] = 0;
    for (int i = 0; i < nl; i++) {
        int n = net.node1[i];
        if (net.direction[i] < 0) n = net.node2[i];
        if (net.nodeType[n] == OUTFALL) {
            n = (net.direction[i] < 0) ? net.node1[i] : net.node2[i];
            net.degree[n]++;
        } else {
            net.degree[n]++;
        }
    }
    // validateGeneralLayout (flowrout.c:274-333)
    std::vector<double> inCount(nn, 0.0);
    for (int j = 0; j < nl; j++) {
        int i = net.node1[j];
        if (net.nodeType[i] != OUTFALL) i = net.node2[j];
        inCount[i] += 1.0;
        // a DUMMY conduit or an ideal pump must be the only link leaving its
        // upstream node (flowrout.c:295-307)
        const bool dummy = net.linkType[j] == CONDUIT && net.xsect[j].type == X_DUMMY;
        const bool ideal = net.linkType[j] == PUMP && net.ncSub[j] == PT_IDEAL;
        if (dummy || ideal) {
            const int u = (net.direction[j] < 0) ? net.node2[j] : net.node1[j];
            if (net.degree[u] > 1) {                  // every offending node is reported
                addError(134, "ERROR 134: Node " + net.nodeId[u] + " has illegal DUMMY link connections.");
                continue;
            }
            // its flow is node_getOutflow of that node (node.c:400-414): a
            // divider's share (divider_getOutflow) is not modelled
            if (net.nodeType[u] == DIVIDER) {
                setError(200, "ERROR 200: a DUMMY conduit or ideal pump leaving Divider " + net.nodeId[u] +
                                  " is not supported by the MI355X engine");
                return;
            }
        }
    }
    if (errorCode) return;
    int outletCount = 0;
    for (int i = 0; i < nn; i++)
        if (net.nodeType[i] == OUTFALL) {
            if (net.degree[i] + (int)inCount[i] > 1) {
                setError(141, "ERROR 141: Outfall " + net.nodeId[i] + " has more than 1 inlet link or an outlet link.");
                return;
            }
            outletCount++;
        }
    if (outletCount == 0) { setError(145, "ERROR 145: drainage system has no acceptable outlet nodes."); return; }
    for (int i = 0; i < nn; i++)
        if (inCount[i] == 0.0) net.degree[i] = -net.degree[i];
    // crown cutoff (dynwave.c:159-160)
    opt.crownCutoff = (opt.surchargeMethod == SUR_SLOT) ? 0.985257 : 0.96;
}

// ===================================================== initial state (start)
// initNodeDepths (flowrout.c:337-385) + link_setOutfallDepth for all links +
// initLinkDepths (flowrout.c:389-421)
void Project::initDepths()
{
    int nn = net.nNodes(), nl = net.nLinks();
    const double* ct = &SWX_CIRC_TABLES[0][0];
    auto geom = [&](int j) {
        const Xsect& x = net.xsect[j];
        return geomOf(x, net.xTab.data());
    };
    State& s = st;
    std::vector<double> acc(nn, 0.0), cnt(nn, 0.0);
    for (int i = 0; i < nl; i++) {
        double y = (s.lNewDepth[i] > kFudge) ? s.lNewDepth[i] + net.offset1[i] : 0.0;
        acc[net.node1[i]] += y; cnt[net.node1[i]] += 1.0;
        acc[net.node2[i]] += y; cnt[net.node2[i]] += 1.0;
    }
    for (int i = 0; i < nn; i++) {
        if (net.nodeType[i] == OUTFALL || net.nodeType[i] == STORAGE) continue;
        if (net.initDepth[i] > 0.0) continue;
        if (cnt[i] > 0.0) s.newDepth[i] = acc[i] / cnt[i];
    }
    for (int i = 0; i < nl; i++) {                  // link_setOutfallDepth for all links
        int k;
        double zz;
        if (net.nodeType[net.node2[i]] == OUTFALL) { k = net.node2[i]; zz = net.offset2[i]; }
        else if (net.nodeType[net.node1[i]] == OUTFALL) { k = net.node1[i]; zz = net.offset1[i]; }
        else continue;
        double yNorm = 0.0, yCrit = 0.0;
        if (net.linkType[i] == CONDUIT) {
            Geom g = geom(i);
            double q = fabs(s.lNewFlow[i] / net.barrels[i]);
            yNorm = linkYnorm(g, q, net.qMax[i], net.beta[i], ct);
            yCrit = getYcrit(g, q, ct);
        }
        // outfall_setOutletDepth (node.c:1413-1492), FREE/NORMAL/FIXED/TSERIES
        double stage, yNew;
        int ot = net.outfallType[k];
        if (ot == O_FREE) { s.newDepth[k] = (zz > 0.0) ? 0.0 : gmin(yNorm, yCrit); continue; }
        if (ot == O_NORMAL) { s.newDepth[k] = (zz > 0.0) ? 0.0 : yNorm; continue; }
        if (ot == O_FIXED) stage = net.fixedStage[k];
        else if (ot == O_TIDAL) {                      // hour 0 of the tide curve
            const Curve& c = net.curves[net.outfallSeries[k]];
            stage = (c.y.empty() ? 0.0 : c.y[0]) / ucfLength();
        }
        else stage = tseriesLookup(net.outfallSeries[k], opt.startDateTime + 0.0 / kMsecPerDay, true) / ucfLength();
        yCrit = gmin(yCrit, yNorm);
        if (yCrit + zz + net.invertElev[k] < stage) yNew = stage - net.invertElev[k];
        else if (zz > 0.0) {
            if (stage < net.invertElev[k] + zz) yNew = gmax(0.0, (stage - net.invertElev[k]));
            else yNew = zz + yCrit;
        } else yNew = yCrit;
        s.newDepth[k] = yNew;
    }
    // initLinkDepths (flowrout.c:389-421)
    for (int i = 0; i < nl; i++) {
        if (net.linkType[i] != CONDUIT || net.q0[i] != 0.0) continue;
        double y1 = s.newDepth[net.node1[i]] - net.offset1[i];
        y1 = gmax(y1, 0.0);
        y1 = gmin(y1, net.xsect[i].yFull);
        double y2 = s.newDepth[net.node2[i]] - net.offset2[i];
        y2 = gmax(y2, 0.0);
        y2 = gmin(y2, net.xsect[i].yFull);
        double y = 0.5 * (y1 + y2);
        y = gmax(y, kFudge);
        s.lNewDepth[i] = y;
    }
}

int Project::initState()
{
    climateInit();                                  // project_init (project.c:295)
    int nn = net.nNodes(), nl = net.nLinks(), P = net.nPollut();
    const double* ct = &SWX_CIRC_TABLES[0][0];
    auto geom = [&](int j) {
        const Xsect& x = net.xsect[j];
        return geomOf(x, net.xTab.data());
    };
    // project_init runs table_tseriesInit before routing_open
    for (auto& ts : net.tseries) {            // table_tseriesInit (table.c:730-740)
        ts.cur = 0;
        ts.x1 = ts.x.empty() ? 0.0 : ts.x[0];
        ts.y1 = ts.y.empty() ? 0.0 : ts.y[0];
        ts.x2 = ts.x1;
        ts.y2 = ts.y1;
        if (ts.x.size() > 1) { ts.cur = 1; ts.x2 = ts.x[1]; ts.y2 = ts.y[1]; }
    }
    State& s = st;
    auto z = [](std::vector<double>& v, int n) { v.assign(n, 0.0); };
    for (auto* v : {&s.newDepth, &s.oldDepth, &s.newVolume, &s.oldVolume, &s.inflow, &s.outflow,
                    &s.overflow, &s.losses, &s.newLatFlow, &s.oldLatFlow, &s.oldNetInflow,
                    &s.oldFlowInflow, &s.oldSurfArea, &s.dYdT, &s.hrt}) z(*v, nn);
    for (auto* v : {&s.lNewFlow, &s.lOldFlow, &s.lNewDepth, &s.lOldDepth, &s.lNewVolume,
                    &s.lOldVolume, &s.surfArea1, &s.surfArea2, &s.froude, &s.dqdh, &s.setting,
                    &s.a1, &s.a2, &s.q1, &s.q2, &s.evapLossRate, &s.seepLossRate}) z(*v, nl);
    s.flowClass.assign(nl, F_DRY);
    s.fullState.assign(nl, 0);
    s.normalFlow.assign(nl, 0);
    s.capacityLimited.assign(nl, 0);
    s.converged.assign(nn, 0);
    z(s.nOldQual, nn * P); z(s.nNewQual, nn * P); z(s.lOldQual, nl * P); z(s.lNewQual, nl * P);
    s.variableStep = 0.0;

    // node_initState (node.c:237-289): junction volume = 0 (fullVolume 0);
    // storage units from their area relation
    for (int j = 0; j < nn; j++) {
        s.oldDepth[j] = net.initDepth[j];
        s.newDepth[j] = s.oldDepth[j];
        net.crownElev[j] = net.invertElev[j];
        if (net.nodeType[j] == STORAGE) {
            net.fullVolume[j] = 0.0;
            net.fullVolume[j] = storageVolume(storageGeom(j), net.fullDepth[j]);
            s.oldVolume[j] = storageVolume(storageGeom(j), s.oldDepth[j]);
        } else {
            net.fullVolume[j] = 0.0;                // node_getVolume(j, fullDepth) = 0
            s.oldVolume[j] = 0.0;
        }
        s.newVolume[j] = s.oldVolume[j];
    }
    // link_initState (link.c:508-539) + conduit_initState (1304-1316) +
    // pump_initState (1534-1544)
    s.targetSetting.assign(nl, 1.0);
    for (auto* v : {&s.ncCOrif, &s.ncCWeir, &s.ncHCrit, &s.ncCSurch}) v->assign(nl, 0.0);
    for (int j = 0; j < nl; j++) {
        s.lOldFlow[j] = net.q0[j];
        s.lNewFlow[j] = net.q0[j];
        s.setting[j] = 1.0;
        if (net.linkType[j] == PUMP) s.setting[j] = s.targetSetting[j] = net.ncInitSetting[j];
        if (net.linkType[j] == CONDUIT) {
            Geom g = geom(j);
            s.lNewDepth[j] = linkYnorm(g, net.q0[j] / net.barrels[j], net.qMax[j], net.beta[j], ct);
        } else {
            s.lNewDepth[j] = 0.0;
            ncCoefs(j);               // orifice / weir coefficients at setting 1 (validation)
        }
        s.lOldDepth[j] = s.lNewDepth[j];
    }
    // hotstart_open (swmm5.c:385) between project_init and routing_open
    bool hot = !hotstartUse.empty();
    if (hot && readHotstart()) return errorCode;
    if (hot) {
        // readRouting's link_setTargetSetting + link_setSetting (hotstart.c:319-322)
        for (int j = 0; j < nl; j++) {
            if (net.linkType[j] == CONDUIT) continue;
            s.targetSetting[j] = s.setting[j];
            if (net.linkType[j] == PUMP) {
                int n1 = net.node1[j];
                if (net.ncYOff[j] > 0.0 && s.setting[j] > 0.0 && s.newDepth[n1] < net.ncYOff[j])
                    s.targetSetting[j] = 0.0;
                if (net.ncYOn[j] > 0.0 && s.setting[j] == 0.0 && s.newDepth[n1] > net.ncYOn[j])
                    s.targetSetting[j] = 1.0;
            }
            s.setting[j] = s.targetSetting[j];
            ncCoefs(j);
        }
    }
    // flowrout_init DW (flowrout.c:75-103): dynwave_init crown elevations
    for (int i = 0; i < nl; i++) {
        int j = net.node1[i];
        double zz = net.invertElev[j] + net.offset1[i] + net.xsect[i].yFull;
        net.crownElev[j] = gmax(net.crownElev[j], zz);
        j = net.node2[i];
        zz = net.invertElev[j] + net.offset2[i] + net.xsect[i].yFull;
        net.crownElev[j] = gmax(net.crownElev[j], zz);
        s.flowClass[i] = F_DRY;
        s.dqdh[i] = 0.0;
    }
    // initNodeDepths / initLinkDepths only without a hot start file (flowrout.c:89-94)
    if (!hot) initDepths();
    // initNodes (flowrout.c:425-468)
    for (int i = 0; i < nn; i++) {
        s.inflow[i] = s.newLatFlow[i];
        s.outflow[i] = 0.0;
        if (opt.allowPonding && net.pondedArea[i] > 0.0 && s.newDepth[i] > net.fullDepth[i])
            s.newVolume[i] = net.fullVolume[i] + (s.newDepth[i] - net.fullDepth[i]) * net.pondedArea[i];
        else
            s.newVolume[i] = (net.fullDepth[i] > 0.0) ? net.fullVolume[i] * (s.newDepth[i] / net.fullDepth[i]) : 0.0;
    }
    for (int i = 0; i < nl; i++) {
        if (s.lNewFlow[i] >= 0.0) {
            s.outflow[net.node1[i]] += s.lNewFlow[i];
            s.inflow[net.node2[i]] += s.lNewFlow[i];
        } else {
            s.inflow[net.node1[i]] -= s.lNewFlow[i];
            s.outflow[net.node2[i]] -= s.lNewFlow[i];
        }
    }
    // initLinks (flowrout.c:472-507)
    for (int i = 0; i < nl; i++) {
        if (net.linkType[i] != CONDUIT) continue;
        s.q1[i] = s.lNewFlow[i] / net.barrels[i];
        s.q2[i] = s.q1[i];
        s.a1[i] = getAofY(geom(i), s.lNewDepth[i], ct);
        s.a2[i] = s.a1[i];
        s.lNewVolume[i] = s.a1[i] * net.lengthT[i] * net.barrels[i];
        s.lOldVolume[i] = s.lNewVolume[i];
    }
    // qualrout_init (qualrout.c:63-96), skipped with a hot start file (routing.c:122)
    for (int p = 0; p < P && !hot; p++) {
        double c0 = net.pollut[p].cInit;
        for (int i = 0; i < nn; i++) {
            double c = (s.newDepth[i] > 0.003281) ? c0 : 0.0;
            s.nOldQual[p * nn + i] = c;
            s.nNewQual[p * nn + i] = c;
        }
        for (int i = 0; i < nl; i++) {
            double c = (s.lNewDepth[i] > 0.003281) ? c0 : 0.0;
            s.lOldQual[p * nl + i] = c;
            s.lNewQual[p * nl + i] = c;
        }
    }
    return 0;
}

// orifice_setSetting / weir_setSetting coefficients at the link's current
// setting (link.c:1729-1765, 2156-2186; weir_validate 2140-2151)
void Project::ncCoefs(int j)
{
    const double* ct = &SWX_CIRC_TABLES[0][0];
    State& s = st;
    NcLink L = ncLink(j);
    const Xsect& x = net.xsect[j];
    Geom g = geomOf(x, net.xTab.data());
    if (net.linkType[j] == ORIFICE) {
        NcCoef c{};
        orificeCoefs(L, g, s.setting[j], ct, &c);
        s.ncCOrif[j] = c.cOrif;
        s.ncCWeir[j] = c.cWeir;
        s.ncHCrit[j] = c.hCrit;
    } else if (net.linkType[j] == WEIR) {
        int cv = net.ncCurve[j];
        const double* cx = cv >= 0 ? net.curves[cv].x.data() : nullptr;
        const double* cy = cv >= 0 ? net.curves[cv].y.data() : nullptr;
        if (!net.ncCanSurcharge[j] && s.ncCSurch[j] != 0.0) return;   // weir_setSetting keeps it
        s.ncCSurch[j] = weirSurchargeCoef(L, g, cx, cy, s.setting[j], ct);
    }
}

NcLink Project::ncLink(int j) const
{
    NcLink L{};
    L.type = net.linkType[j];
    L.sub = net.ncSub[j];
    L.flap = net.hasFlapGate[j];
    L.canSurcharge = net.ncCanSurcharge[j];
    int cv = net.ncCurve[j];
    L.cOff = 0;
    L.cN = cv >= 0 ? (int)net.curves[cv].x.size() : 0;
    L.offset1 = net.offset1[j];
    L.yFull = net.xsect[j].yFull;
    L.c1 = net.ncC1[j];
    L.c2 = net.ncC2[j];
    L.endCon = net.ncEndCon[j];
    L.slope = net.ncSlope[j];
    L.length = net.ncLength[j];
    L.yOn = net.ncYOn[j];
    L.yOff = net.ncYOff[j];
    L.xMin = net.ncXMin[j];
    L.xMax = net.ncXMax[j];
    L.qFull = net.qFull[j];
    L.ucfL = ucfLength();
    L.ucfQ = ucfFlow();
    L.si = opt.unitSystem;
    L.roadWidth = net.ncRoadWidth[j];
    L.roadSurf = net.ncRoadSurf[j];
    L.qLimit = net.qLimit[j];
    return L;
}

StorageGeom Project::storageGeom(int j) const
{
    StorageGeom g;
    g.shape = net.stShape[j];
    g.a0 = net.stA0[j];
    g.a1 = net.stA1[j];
    g.a2 = net.stA2[j];
    int c = net.stCurve[j];
    g.cx = (c >= 0 && !net.curves[c].x.empty()) ? net.curves[c].x.data() : nullptr;
    g.cy = (c >= 0 && !net.curves[c].y.empty()) ? net.curves[c].y.data() : nullptr;
    g.cn = (c >= 0) ? (int)net.curves[c].x.size() : 0;
    g.fullDepth = net.fullDepth[j];
    g.fullVolume = net.fullVolume[j];
    g.ucfL = ucfLength();
    g.ucfV = ucfVolume();
    return g;
}

// ================================================================= inflows
double Project::getDateTime(double elapsedMsec) const
{
    return addSeconds(opt.startDateTime, (elapsedMsec + 1) / 1000.0);
}

// climate_validate (climate.c:480-527): a climate file where evaporation or
// wind needs one (ERROR 336), opened and positioned (climate_openFile:
// 337-339), the snow melt parameters (181), then the monthly temperature
// adjustments in deg F and the evaporation adjustments in ft/s.  The errors
// are reported and validation goes on, as report_writeErrorMsg does.
void Project::climateValidate()
{
    if ((opt.windFile || opt.evapType == 3 || opt.evapType == 4) && opt.climateFile.empty())
        addError(336, "ERROR 336: no climate file specified for evaporation and/or wind speed.");
    if (!opt.climateFile.empty()) {
        climFile_.reset(new ClimateFile());
        climFile_->open(opt.climateFile, opt.startDate, opt.climateStart, opt.climateUnits, opt.unitSystem == 1,
                        opt.airTemp, errorCode == 0);
        for (int c : climFile_->errors) {
            const char* what = c == 337 ? "cannot open climate file " : c == 338 ? "error in reading from climate file "
                                                                                 : "attempt to read beyond end of climate file ";
            addError(c, "ERROR " + std::to_string(c) + ": " + what + opt.climateFile + ".");
        }
        climErrSeen_ = climFile_->errors.size();
    }
    if (opt.snowTipm < 0.0 || opt.snowTipm > 1.0 || opt.snowRnm < 0.0 || opt.snowRnm > 1.0)
        addError(181, "ERROR 181: invalid snow melt climatology parameters.");
    if (opt.anglat <= -89.99 || opt.anglat >= 89.99) addError(181, "ERROR 181: invalid snow melt climatology parameters.");
    for (int i = 0; i < 12; i++) {
        if (opt.unitSystem == 1) opt.adjustTemp[i] *= 9.0 / 5.0;
        opt.adjustEvap[i] /= ucfEvapRate();
    }
}

// climate_initState (climate.c:598-637), the evaporation part.  StartDate
// is the start's date without its time of day, as in the reference.
void Project::climateInit()
{
    lastTempDay_ = -693594;                        // LastDay = NO_DATE
    if (opt.evapType == 3) tempEvap_.reset();
    nextEvapDate_ = opt.startDate;
    nextEvapRate_ = 0.0;
    evapCursor_ = 0;
    if (opt.evapType == 2 && opt.evapSeries >= 0) {
        const Tseries& t = net.tseries[opt.evapSeries];
        if (!t.x.empty()) {                        // table_getFirstEntry
            nextEvapDate_ = t.x[0];
            nextEvapRate_ = t.y[0];
            evapCursor_ = 0;
        }
        if (nextEvapDate_ < opt.startDate) setNextEvapDate(opt.startDate);
        opt.evapRate = nextEvapRate_ / ucfEvapRate();
        setNextEvapDate(nextEvapDate_);
        // project_init then runs table_tseriesInit on every series
        // (project.c:297): the cursor goes to the series' second entry
        evapCursor_ = (t.x.size() > 1) ? 1 : 0;
    }
}

// setNextEvapDate (climate.c:671-725): CONSTANT, MONTHLY, TIMESERIES
void Project::setNextEvapDate(double theDate)
{
    if (nextEvapDate_ > theDate) return;
    switch (opt.evapType) {
    case 0:
        nextEvapDate_ = theDate + 365.;
        break;
    case 1: {
        int yr, mon, day;
        decodeDate(theDate, &yr, &mon, &day);
        if (mon == 12) { mon = 1; yr++; }
        else mon++;
        nextEvapDate_ = encodeDate(yr, mon, 1);
        break;
    }
    case 3:
        nextEvapDate_ = theDate + 365.;
        break;
    case 4:                                        // climate file: the next day
        nextEvapDate_ = floor(theDate) + 1.0;
        break;
    default:
        if (opt.evapSeries >= 0) {
            const Tseries& t = net.tseries[opt.evapSeries];
            nextEvapDate_ = theDate + 365.;
            // table_getNextEntry from the cursor, entries up to EndDateTime
            while (evapCursor_ + 1 < t.x.size() && t.x[evapCursor_ + 1] <= opt.endDateTime) {
                evapCursor_++;
                const double d = t.x[evapCursor_], e = t.y[evapCursor_];
                if (d >= theDate) {
                    nextEvapDate_ = d;
                    nextEvapRate_ = e;
                    break;
                }
            }
        }
        break;
    }
}

// climate_setState (climate.c:641-655) -> setEvap (876-911): the rate for the
// routing step starting at theDate (swmm5.c:556 without runoff)
double Project::climateSetState(double theDate)
{
    const int mon = monthOfYear(theDate);
    // updateFileValues (climate.c:734-778); a read error ends the run
    if (climFile_) {
        climFile_->update(theDate, opt.startDateTime);
        for (; climErrSeen_ < climFile_->errors.size(); climErrSeen_++)
            setError(338, "ERROR 338: error in reading from climate file " + opt.climateFile + ".");
    }
    // setTemp (climate.c:782-831): with the climate file's temperatures, a
    // new day's min / max (adjusted, ordered) feed the temperature
    // evaporation's moving averages; LastDay is the date of that call
    if (opt.tempSource == 2 && climFile_ && floor(theDate) > lastTempDay_) {
        double tmin = climFile_->value[ClimateFile::TMIN] + opt.adjustTemp[mon - 1];
        double tmax = climFile_->value[ClimateFile::TMAX] + opt.adjustTemp[mon - 1];
        if (tmin > tmax) std::swap(tmin, tmax);
        if (opt.evapType == 3)
            climFile_->value[ClimateFile::EVAP] = tempEvap_.day(dayOfYear(theDate), tmin, tmax, opt.anglat,
                                                               opt.unitSystem == 1);
        lastTempDay_ = theDate;
    }
    switch (opt.evapType) {
    case 0: opt.evapRate = opt.monthlyEvap[0] / ucfEvapRate(); break;
    case 1: opt.evapRate = opt.monthlyEvap[mon - 1] / ucfEvapRate(); break;
    case 3:                                        // TEMPERATURE (climate.c:902-904)
        opt.evapRate = (climFile_ ? climFile_->value[ClimateFile::EVAP] : 0.0) / ucfEvapRate();
        break;
    case 4:                                        // FILE (climate.c:897-900)
        opt.evapRate = (climFile_ ? climFile_->value[ClimateFile::EVAP] : 0.0) / ucfEvapRate();
        opt.evapRate *= opt.panCoeff[mon - 1];
        break;
    default:
        if (theDate >= nextEvapDate_) opt.evapRate = nextEvapRate_ / ucfEvapRate();
        break;
    }
    // the climate change adjustment is added at every call (for a time series
    // the unrefreshed rate keeps the earlier additions, as in the reference)
    opt.evapRate += opt.adjustEvap[mon - 1];
    // soil recovery factor (setEvap, climate.c:913-918) and the conductivity
    // adjustment (climate_setState, climate.c:653): storage exfiltration and
    // conduit seepage
    opt.recoveryFactor = 1.0;
    const int rp = opt.evapRecovery;
    if (rp >= 0 && net.patterns[rp].type == PAT_MONTHLY) opt.recoveryFactor = net.patterns[rp].factor[mon - 1];
    opt.hydconFactor = opt.adjustHydcon[mon - 1];
    setNextEvapDate(theDate);
    return opt.evapRate;
}

bool Project::evapCanBePositive() const
{
    bool adj = false;
    for (double a : opt.adjustEvap) adj = adj || a != 0.0;
    if (opt.evapType == 0) return opt.evapRate > 0.0 || adj;
    if (opt.evapType == 3 || opt.evapType == 4) return true;    // climate file: any day may evaporate
    if (opt.evapType == 1) {
        for (double m : opt.monthlyEvap) adj = adj || m > 0.0;
        return adj;
    }
    if (opt.evapSeries >= 0)
        for (double y : net.tseries[opt.evapSeries].y) adj = adj || y > 0.0;
    return adj;
}

double Project::patternFactor(int p, int month, int day, int hour) const  // inflow.c:456-484
{
    const Pattern& pt = net.patterns[p];
    switch (pt.type) {
    case PAT_MONTHLY: if (month >= 0 && month < 12) return pt.factor[month]; break;
    case PAT_DAILY: if (day >= 0 && day < 7) return pt.factor[day]; break;
    case PAT_HOURLY: if (hour >= 0 && hour < 24) return pt.factor[hour]; break;
    case PAT_WEEKEND:
        if (day == 0 || day == 6)
            if (hour >= 0 && hour < 24) return pt.factor[hour];
        break;
    }
    return 1.0;
}

// table.c:745-806 (in-memory series)
double Project::tseriesLookup(int k, double x, bool extend)
{
    Tseries& t = net.tseries[k];
    auto interp = [](double xx, double x1, double y1, double x2, double y2) {
        double dx = x2 - x1;
        if (fabs(dx) < 1.0e-20) return (y1 + y2) / 2.;
        return y1 + (xx - x1) * (y2 - y1) / dx;
    };
    if (t.x1 <= x && t.x2 >= x && t.x1 != t.x2) return interp(x, t.x1, t.y1, t.x2, t.y2);
    if (t.x1 == t.x2 || x < t.x1) {
        t.cur = 0;
        t.x1 = t.x.empty() ? 0.0 : t.x[0];
        t.y1 = t.y.empty() ? 0.0 : t.y[0];
        if (x < t.x1) return extend ? t.y1 : 0.0;
    }
    t.x1 = t.x2;
    t.y1 = t.y2;
    while (t.cur + 1 < t.x.size()) {
        t.cur++;
        t.x2 = t.x[t.cur];
        t.y2 = t.y[t.cur];
        if (x <= t.x2) return interp(x, t.x1, t.y1, t.x2, t.y2);
        t.x1 = t.x2;
        t.y1 = t.y2;
    }
    return extend ? t.y1 : 0.0;
}

bool Project::inflowsAreConstant() const
{
    if (!net.extInflows.empty()) return false;
    for (auto& d : net.dwfInflows)
        for (int i = 0; i < 4; i++)
            if (d.patterns[i] >= 0) return false;
    return true;
}

void Project::evalInflows(double currentDate, std::vector<double>& lat,
                          std::vector<double>* qual, double* dwfTotal, double* extTotal,
                          double* extOut)
{
    int nn = net.nNodes(), P = net.nPollut();
    lat.assign(nn, 0.0);
    if (qual) qual->assign((size_t)nn * P, 0.0);
    double dwf = 0.0, ext = 0.0, eout = 0.0;
    // addExternalInflows (routing.c:435-494): per node, FLOW first then pollutants
    std::vector<int> extFirst(nn, -1);
    std::vector<int> order(net.extInflows.size());
    // the reference keeps each node's inflows in a prepended list: last read first
    std::vector<std::vector<int>> byNode(nn);
    for (int i = 0; i < (int)net.extInflows.size(); i++) byNode[net.extInflows[i].node].push_back(i);
    int month = -1, day = -1, hour = -1;
    auto extValue = [&](const ExtInflow& in) {   // inflow.c:207-230
        double blv = in.baseline, tsv = 0.0;
        if (in.basePat >= 0) {
            if (month < 0) { month = monthOfYear(currentDate) - 1; day = dayOfWeek(currentDate) - 1; hour = hourOfDay(currentDate); }
            blv *= patternFactor(in.basePat, month, day, hour);
        }
        if (in.tseries >= 0) tsv = tseriesLookup(in.tseries, currentDate, false) * in.sFactor;
        return in.cFactor * (tsv + blv);
    };
    for (int j = 0; j < nn; j++) {
        if (byNode[j].empty()) continue;
        double q = 0.0;
        for (int k = (int)byNode[j].size() - 1; k >= 0; k--) {
            const ExtInflow& in = net.extInflows[byNode[j][k]];
            if (in.type == EXT_FLOW) { q += extValue(in); break; }
        }
        if (fabs(q) < kFlowTol) q = 0.0;
        lat[j] += q;
        if (q >= 0.0) ext += q;
        else { eout += -q; continue; }
        if (net.nodeType[j] == OUTFALL && st.oldNetInflow[j] < 0.0) q = q - st.oldNetInflow[j];
        if (qual)
            for (int k = (int)byNode[j].size() - 1; k >= 0; k--) {
                const ExtInflow& in = net.extInflows[byNode[j][k]];
                if (in.type == EXT_FLOW) continue;
                double w = extValue(in);
                if (in.type == EXT_CONCEN) w *= q;
                (*qual)[(size_t)in.param * nn + j] += w;
            }
    }
    // addDryWeatherInflows (routing.c:498-575)
    month = monthOfYear(currentDate) - 1;
    day = dayOfWeek(currentDate) - 1;
    hour = hourOfDay(currentDate);
    std::vector<std::vector<int>> dwfByNode(nn);
    for (int i = 0; i < (int)net.dwfInflows.size(); i++) dwfByNode[net.dwfInflows[i].node].push_back(i);
    auto dwfValue = [&](const DwfInflow& in) {   // inflow.c:361-390
        double f = 1.0;
        int p1 = in.patterns[PAT_MONTHLY];
        if (p1 >= 0) f *= patternFactor(p1, month, day, hour);
        p1 = in.patterns[PAT_DAILY];
        if (p1 >= 0) f *= patternFactor(p1, month, day, hour);
        p1 = in.patterns[PAT_HOURLY];
        int p2 = in.patterns[PAT_WEEKEND];
        if (p2 >= 0) {
            if (day == 0 || day == 6) f *= patternFactor(p2, month, day, hour);
            else if (p1 >= 0) f *= patternFactor(p1, month, day, hour);
        } else if (p1 >= 0) f *= patternFactor(p1, month, day, hour);
        return f * in.avgValue;
    };
    for (int j = 0; j < nn; j++) {
        if (dwfByNode[j].empty()) continue;
        double q = 0.0;
        for (int k = (int)dwfByNode[j].size() - 1; k >= 0; k--) {
            const DwfInflow& in = net.dwfInflows[dwfByNode[j][k]];
            if (in.param < 0) { q = dwfValue(in); break; }
        }
        if (fabs(q) < kFlowTol) q = 0.0;
        lat[j] += q;
        dwf += q;
        if (q <= 0.0 || !qual) continue;
        for (int p = 0; p < P; p++)
            if (net.pollut[p].cDWF > 0.0) (*qual)[(size_t)p * nn + j] += q * net.pollut[p].cDWF;
        for (int k = (int)dwfByNode[j].size() - 1; k >= 0; k--) {
            const DwfInflow& in = net.dwfInflows[dwfByNode[j][k]];
            if (in.param < 0) continue;
            int p = in.param;
            (*qual)[(size_t)p * nn + j] += q * dwfValue(in);
            if (net.pollut[p].cDWF > 0.0) (*qual)[(size_t)p * nn + j] -= q * net.pollut[p].cDWF;
        }
    }
    if (dwfTotal) *dwfTotal = dwf;
    if (extTotal) *extTotal = ext;
    if (extOut) *extOut = eout;
}

}  // namespace swx
