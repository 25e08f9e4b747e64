/* ref_timing.c -- TEST INFRASTRUCTURE ONLY: times the reference EPA SWMM 5.2.4
 * solver itself (oracle/_ref/libswmm5_ref.so, compiled from /root/reference's
 * own sources by oracle/Makefile) on an input file, for bench.py's
 * cpu_baseline leg.  The harness is SURVEY.md Appendix B's:
 *     swmm_open; swmm_start(0); clock around swmm_step until the sample ends
 * (at most maxSeconds of stepping or maxSteps steps, or the end of the run),
 * then swmm_end / swmm_close, which write the report whose "Average
 * Iterations per Step" (stats.c TimeStepStats over exactly the stepped
 * steps) gives the Picard iterations.  The thread count is the input's
 * THREADS option (project.c:689-693).  Prints one JSON object.
 *   usage: ref_timing INP RPT OUT MAX_SECONDS MAX_STEPS
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "swmm5.h"

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char** argv)
{
    if (argc < 6) {
        fprintf(stderr, "usage: %s INP RPT OUT MAX_SECONDS MAX_STEPS\n", argv[0]);
        return 2;
    }
    const double maxSec = atof(argv[4]);
    const long maxSteps = atol(argv[5]);
    double t0 = now();
    int err = swmm_open(argv[1], argv[2], argv[3]);
    double t1 = now();
    if (!err) err = swmm_start(0);
    double t2 = now();
    long steps = 0;
    double elapsed = 0.0, t3 = t2;
    if (!err) {
        do {
            err = swmm_step(&elapsed);
            steps++;
            t3 = now();
        } while (!err && elapsed > 0.0 && t3 - t2 < maxSec && steps < maxSteps);
    }
    int nlinks = swmm_getCount(swmm_LINK);
    swmm_end();
    swmm_close();
    /* Routing Time Step Summary: "Average Iterations per Step : x" */
    double iters = -1.0;
    FILE* f = fopen(argv[2], "r");
    if (f) {
        char line[512];
        while (fgets(line, sizeof line, f)) {
            char* p = strstr(line, "Average Iterations per Step");
            if (p && (p = strchr(p, ':'))) iters = atof(p + 1);
        }
        fclose(f);
    }
    printf("{\"error\": %d, \"open_s\": %.3f, \"start_s\": %.3f, \"steps\": %ld, \"step_s\": %.4f, "
           "\"links\": %d, \"iterations_per_step\": %.3f}\n",
           err, t1 - t0, t2 - t1, steps, t3 - t2, nlinks, iters);
    return err ? 1 : 0;
}
