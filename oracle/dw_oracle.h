/*
 * dw_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of EPA SWMM 5.2.4's dynamic-wave routing step, written in
 * plain C over structure-of-arrays state.  It is the parity checker for the
 * MI355X path (tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg only); nothing in the product links or calls it.  It is pinned against
 * the reference itself: tests/test_oracle_vs_reference.py replays reference
 * runs captured by oracle/refdump.c (compiled from /root/reference) and
 * requires bit-identical state after every routing step.
 *
 * Scope: junctions + outfalls (FREE / NORMAL / FIXED), conduits of shape
 * CIRCULAR, RECT_OPEN, RECT_CLOSED, TRAPEZOIDAL, TRIANGULAR; EXTRAN and SLOT
 * surcharge; ponding; local losses; flap gates; seepage/evaporation losses;
 * variable (Courant) time step; pollutant advection (qualrout.c).
 */
#ifndef DW_ORACLE_H
#define DW_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_net orc_net;

orc_net* orc_alloc(int nNodes, int nLinks, int nPollut);
void     orc_free(orc_net* net);
/* Pointer to a named fp64 / int32 array (NULL if unknown). */
double*  orc_fd(orc_net* net, const char* name);
int*     orc_fi(orc_net* net, const char* name);
/* Named scalar options (see dw_oracle.c: OPTION TABLE). */
int      orc_set_opt(orc_net* net, const char* name, double value);
double   orc_get_opt(orc_net* net, const char* name);
/* Finish setup after static arrays are filled: derives isTrueConduit etc. */
int      orc_prepare(orc_net* net);
/* dynwave_getRoutingStep (dynwave.c:195-220) */
double   orc_routing_step(orc_net* net, double fixedStep);
/* One routing step with lateral inflows already placed in "latIn"
 * (and pollutant mass loads in "qualIn", P x nNodes).  Returns Picard
 * iterations (dynwave_execute's Steps). */
int      orc_step(orc_net* net, double dt);
/* Single-function known-answer hooks: fn = 0 AofY, 1 WofY, 2 RofY, 3 YofA,
 * 4 AofS, 5 Ycrit, 6 Ynorm(q), 7 SofA, 8 dSdA, 9 Froude(v=x, y=x2) */
double   orc_xsect(orc_net* net, int fn, int link, double x, double x2);

#ifdef __cplusplus
}
#endif
#endif
