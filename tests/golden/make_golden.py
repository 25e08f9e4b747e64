"""Regenerate the golden fixtures from the compiled reference.

TEST INFRASTRUCTURE ONLY -- needs /root/reference (the oracle/_ref build); run
in the survey container, never on the GPU box:

    make -C oracle ref && python tests/golden/make_golden.py

For every case it writes the input file (<case>.inp, produced by the
deterministic generators in stormwater-management-model_amd/netgen.py) and
<case>.npz: the reference's static parameters, its state right after
swmm_start and its full-precision state after every `every`-th routing step
(oracle/refdump.c reads them from the reference's exported globals), plus
the run statistics (NodeStats / LinkStats / OutfallStats, "st.*") after the
last step, the reference's binary results (<case>.ref_out.npy) and its report
file (<case>.ref_rpt.txt) and, for a case that saves a hot start file, that
file (<case>.ref.hsf).
"""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "stormwater-management-model_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import netgen  # noqa: E402
from _dumpio import read_dump  # noqa: E402

REFDUMP = os.path.join(ROOT, "oracle", "_ref", "refdump")
REFDUMP_FMA = os.path.join(ROOT, "oracle", "_ref", "fma", "refdump")
REFDUMP_X87 = os.path.join(ROOT, "oracle", "_ref", "x87", "refdump")
# cases whose results are ill-conditioned in the reference itself (non-basic
# shapes at outfalls: Newton A(S) with a 1e-4 stopping tolerance, critical
# depth by enumeration): the fixture also stores, per recorded step and state
# array, the largest |FMA build - reference| ("env.<key>"), made with
# `make -C oracle ref-fma`
ENVELOPE = {"example_shapes", "example_shapes_var", "example_irregular", "example_irregular_var",
            "example_culverts", "example_culverts_var", "example_streets", "example_branches",
            "example_branches_var", "example_dummy", "example_dummy_var"}

# envelope cases whose report tables also carry the x87 build's report (the
# report test then accepts twice the larger of the two builds' differences)
X87_RPT = {"example_branches", "example_branches_var"}

# name -> (writer, kwargs, every)
CASES = {
    "grid12": (netgen.write_grid, dict(nx=12, ny=12, end_time="00:10:00"), 4),
    "grid12_var_qual": (netgen.write_grid, dict(nx=12, ny=12, end_time="00:20:00",
                                                variable_step=0.75, route_step=5,
                                                pollutants=3), 2),
    "grid10_surcharge": (netgen.write_grid, dict(nx=10, ny=10, end_time="00:40:00",
                                                 variable_step=0.75, route_step=5,
                                                 diameter=1.0, q=0.1), 3),
    "example": (netgen.write_example, dict(end_time="02:00:00", route_step=5.0), 1),
    "example_var": (netgen.write_example, dict(end_time="02:00:00", route_step=10.0,
                                               variable_step=0.75), 1),
    "example_qual": (netgen.write_example, dict(end_time="01:00:00", route_step=5.0,
                                                pollutants=True), 1),
    # hot start: the first run saves its final state, the second starts from
    # the reference's saved file (kept as example_hotsave.ref.hsf)
    "example_hotsave": (netgen.write_example, dict(end_time="01:00:00", route_step=5.0,
                                                   pollutants=True,
                                                   files="SAVE HOTSTART example_hotsave.hsf"), 1),
    "example_hot": (netgen.write_example, dict(end_time="01:00:00", route_step=5.0,
                                               pollutants=True,
                                               files="USE HOTSTART example_hotsave.ref.hsf"), 1),
    # storage units of every area relation, evaporation (node.c:654-1105)
    "example_storage": (netgen.write_example, dict(end_time="02:00:00", route_step=5.0,
                                                   storage=True), 1),
    "example_storage_var": (netgen.write_example, dict(end_time="02:00:00", route_step=10.0,
                                                       variable_step=0.75, storage=True), 1),
    "example_storage_qual": (netgen.write_example, dict(end_time="01:30:00", route_step=5.0,
                                                        storage=True, pollutants=True), 1),
    # pumps of every curve type, orifices, weirs, outlets (link.c:1406-2692)
    "example_regulators": (netgen.write_example, dict(end_time="02:00:00", route_step=5.0,
                                                      regulators=True), 1),
    "example_regulators_var_qual": (netgen.write_example, dict(end_time="01:30:00", route_step=10.0,
                                                               variable_step=0.75, regulators=True,
                                                               pollutants=True), 1),
    # every non-basic cross-section shape (xsect.c:216-2618) and a force main,
    # fixed step / variable step with Darcy-Weisbach force-main friction
    "example_shapes": (netgen.write_example, dict(end_time="02:00:00", route_step=5.0,
                                                  shapes=True), 1),
    "example_shapes_var": (netgen.write_example, dict(end_time="02:00:00", route_step=10.0,
                                                      variable_step=0.75, shapes=True,
                                                      force_main_eqn="D-W", pollutants=True), 1),
    # irregular transects (overbanks, meander factor, station / elevation
    # adjustments) and custom shape curves (transect.c, shape.c)
    "example_irregular": (netgen.write_example, dict(end_time="02:00:00", route_step=5.0,
                                                     irregular=True), 1),
    "example_irregular_var": (netgen.write_example, dict(end_time="02:00:00", route_step=10.0,
                                                         variable_step=0.75, irregular=True,
                                                         pollutants=True), 1),
    # culverts under inlet control (culvert.c): both equation forms
    "example_culverts": (netgen.write_example, dict(end_time="02:00:00", route_step=5.0,
                                                    culverts=True), 1),
    "example_culverts_var": (netgen.write_example, dict(end_time="02:00:00", route_step=10.0,
                                                        variable_step=0.75, culverts=True), 1),
    # tidal-curve and stage-time-series outfalls (node.c:1446-1459)
    "example_tidal": (netgen.write_example, dict(end_time="03:00:00", route_step=5.0, tidal=True), 1),
    "example_tidal_var": (netgen.write_example, dict(end_time="03:00:00", route_step=10.0,
                                                     variable_step=0.75, tidal=True), 1),
    # roadway weirs (roadway.c)
    "example_roadway": (netgen.write_example, dict(end_time="02:00:00", route_step=5.0, roadway=True), 1),
    # flow dividers (routed as junctions under dynamic wave)
    "example_dividers": (netgen.write_example, dict(end_time="02:00:00", route_step=5.0, dividers=True,
                                                    pollutants=True), 1),
    # street cross sections (street.c)
    "example_streets": (netgen.write_example, dict(end_time="02:00:00", route_step=5.0, streets=True), 1),
    # inflow hydrograph from an external time series file
    "example_extfile": (netgen.write_example, dict(end_time="02:00:00", route_step=5.0, extfile=True), 1),
    # every flow class (dwflow.c:297-413): backwater over an invert offset and
    # a weir crest (UP_CRITICAL), a depth-curve pump below its curve (DN_DRY)
    "example_branches": (netgen.write_example, dict(end_time="01:40:00", route_step=5.0, branches=True), 1),
    "example_evap_monthly": (netgen.write_example, dict(end_time="01:00:00", route_step=5.0, storage=True,
                                                        evap="MONTHLY"), 1),
    "example_evap_series": (netgen.write_example, dict(end_time="01:00:00", route_step=10.0,
                                                       variable_step=0.75, storage=True, evap="TIMESERIES"), 1),
    # REPORT AVERAGES (output.c:857-955): each period's average of the routing
    # steps' results, pumps and regulators keeping their current setting
    "example_avg": (netgen.write_example, dict(end_time="01:30:00", route_step=10.0, variable_step=0.75,
                                               regulators=True, pollutants=True, averages=True), 1),
    # storage seepage (exfil.c: Green-Ampt bottom and banks, constant rate),
    # conduit seepage, CONDUCTIVITY adjustments and an evaporation RECOVERY
    # pattern across a month boundary (climate.c:641-655, 895-918)
    "example_exfil": (netgen.write_example, dict(end_time="01:30:00", route_step=5.0, exfil=True,
                                                 pollutants=True), 1),
    "example_exfil_var": (netgen.write_example, dict(end_time="01:30:00", route_step=10.0,
                                                     variable_step=0.75, exfil=True), 1),
    # climate-file evaporation (climate.c:531-1619): daily pan evaporation
    # times monthly pan coefficients, and Hargreaves evaporation from daily
    # temperatures with its 7-day moving averages, from each of the four
    # climate file formats, over two midnights and the month boundary
    "example_evap_file": (netgen.write_example, dict(end_time="02:00:00", route_step=30.0, storage=True,
                                                     evap="FILE:USER", options={"REPORT_STEP": "01:00:00"}), 10),
    "example_evap_temp": (netgen.write_example, dict(end_time="02:00:00", route_step=30.0, storage=True,
                                                     evap="TEMPERATURE:GHCND", options={"REPORT_STEP": "01:00:00"}), 10),
    "example_evap_td3200": (netgen.write_example, dict(end_time="02:00:00", route_step=30.0, storage=True,
                                                       evap="FILE:TD3200", options={"REPORT_STEP": "01:00:00"}), 10),
    "example_evap_dly": (netgen.write_example, dict(end_time="02:00:00", route_step=30.0, storage=True,
                                                    evap="TEMPERATURE:DLY0204", options={"REPORT_STEP": "01:00:00"}), 10),
    # SKIP_STEADY_STATE (routing.c:236-244, 383-395): the hydrograph passes,
    # the system settles and steps are skipped while the inflows and the
    # step's flow error stay within LAT_FLOW_TOL / SYS_FLOW_TOL
    "example_steady": (netgen.write_example, dict(end_time="08:00:00", route_step=10.0,
                                                  options={"SKIP_STEADY_STATE": "YES"}), 2),
    "example_steady_var": (netgen.write_example, dict(end_time="08:00:00", route_step=10.0,
                                                      variable_step=0.75,
                                                      options={"SKIP_STEADY_STATE": "YES",
                                                               "SYS_FLOW_TOL": "1",
                                                               "LAT_FLOW_TOL": "2"}), 2),
    # SKIP_STEADY_STATE with pumps (C17 switches on above 2.0 ft and off
    # below 0.5 ft of its inlet depth: a step whose pump settings change is
    # never steady, routing.c:224, 388-391), storage units and pollutants
    "example_steady_pump": (netgen.write_example, dict(end_time="08:00:00", route_step=10.0,
                                                       regulators=True, storage=True, pollutants=True,
                                                       options={"SKIP_STEADY_STATE": "YES"}), 1),
    "example_dummy": (netgen.write_example, dict(end_time="02:00:00", route_step=5.0, dummy=True,
                                                 pollutants=True), 1),
    "example_dummy_var": (netgen.write_example, dict(end_time="02:00:00", route_step=10.0, variable_step=0.75,
                                                     dummy=True), 1),
    "example_branches_var": (netgen.write_example, dict(end_time="01:40:00", route_step=10.0,
                                                        variable_step=0.75, branches=True,
                                                        options={"INERTIAL_DAMPING": "NONE"}), 1),
    # Preissmann slot surcharge (dwflow.c:575-588, dynwave.c:159), ponding
    # (dynwave.c:309, 661, 766-795), full inertial damping, slope-only
    # normal-flow limitation
    "example_slot_pond": (netgen.write_example, dict(end_time="01:40:00", route_step=5.0, ponding=True,
                                                     options={"SURCHARGE_METHOD": "SLOT",
                                                              "ALLOW_PONDING": "YES",
                                                              "NORMAL_FLOW_LIMITED": "SLOPE",
                                                              "INERTIAL_DAMPING": "FULL"}), 1),
    # no inertial damping, Froude-only normal-flow limitation, conduit
    # lengthening (link.c:1104-1118, 1217-1254), ponding under EXTRAN
    "example_options": (netgen.write_example, dict(end_time="01:40:00", route_step=30.0,
                                                   variable_step=0.75, ponding=True,
                                                   options={"ALLOW_PONDING": "YES",
                                                            "INERTIAL_DAMPING": "NONE",
                                                            "NORMAL_FLOW_LIMITED": "FROUDE",
                                                            "LENGTHENING_STEP": "60"}), 1),
    # the surcharged grid under the slot method, no normal-flow limitation
    "grid10_slot": (netgen.write_grid, dict(nx=10, ny=10, end_time="00:40:00", variable_step=0.75,
                                            route_step=5, diameter=1.0, q=0.1,
                                            extra_options=("SURCHARGE_METHOD SLOT",
                                                           "NORMAL_FLOW_LIMITED NONE",
                                                           "INERTIAL_DAMPING NONE")), 3),
    # swmm_setValue between steps: external inflow, outfall stage, routing step
    "example_api": (netgen.write_example, dict(end_time="01:00:00", route_step=10.0,
                                               variable_step=0.75), 1),
    # swmm_stride calls shorter and longer than the routing step (swmm5.c:466-510)
    "example_stride": (netgen.write_example, dict(end_time="01:00:00", route_step=60.0,
                                                  variable_step=0.75), 1),
    "example_stride_fixed": (netgen.write_example, dict(end_time="01:00:00", route_step=10.0), 1),
}
# REFDUMP_ACTIONS per case: "afterStep:property:object:value" (swmm5.h codes)
ACTIONS = {
    "example_api": "40:306:N3:2.5;90:304:O1:104.2;150:3:-:4.0;200:306:N3:0.0;260:304:O2:104.5",
    "example_stride": "10:-1:-:3;11:-1:-:7;12:-1:-:45;30:-1:-:25;31:-1:-:2;50:-1:-:1;51:-1:-:90",
    "example_stride_fixed": "20:-1:-:3;21:-1:-:7;40:-1:-:25;41:-1:-:4",
}


def make(name):
    writer, kw, every = CASES[name]
    inp = os.path.join(HERE, name + ".inp")
    if writer is netgen.write_grid:
        kw = dict(kw)
        nx, ny = kw.pop("nx"), kw.pop("ny")
        writer(inp, nx, ny, **kw)
    else:
        writer(inp, **kw)
    tmp = "/tmp/golden_" + name
    env = dict(os.environ)
    if name in ACTIONS:
        env["REFDUMP_ACTIONS"] = ACTIONS[name]
    subprocess.run([REFDUMP, inp, tmp + ".rpt", tmp + ".out", tmp + ".bin", "0", str(every)],
                   check=True, stdout=subprocess.DEVNULL, env=env)
    d = read_dump(tmp + ".bin")
    if name in ENVELOPE:
        subprocess.run([REFDUMP_FMA, inp, tmp + "_fma.rpt", tmp + "_fma.out", tmp + "_fma.bin", "0",
                        str(every)], check=True, stdout=subprocess.DEVNULL, env=env)
        e = read_dump(tmp + "_fma.bin")
        subprocess.run([REFDUMP_X87, inp, tmp + "_x87.rpt", tmp + "_x87.out", tmp + "_x87.bin", "0",
                        str(every)], check=True, stdout=subprocess.DEVNULL, env=env)
        x = read_dump(tmp + "_x87.bin")
        for k in list(d):
            if k.startswith("s.") and k in e and d[k].ndim == 2 and d[k].dtype == np.float64 \
                    and d[k].shape == e[k].shape:
                env_k = np.abs(d[k] - e[k]).max(axis=1)
                if k in x and x[k].ndim == 2:           # x87 may take another number of steps
                    n = min(len(x[k]), len(d[k]))
                    ex = np.abs(d[k][:n] - x[k][:n]).max(axis=1)
                    env_k[:n] = np.maximum(env_k[:n], ex)
                    env_k[n:] = np.maximum(env_k[n:], ex.max())
                d["env." + k[2:]] = env_k
            elif k.startswith("st.") and k in e and d[k].shape == e[k].shape:
                env_k = np.abs(d[k].astype(np.float64) - e[k].astype(np.float64))
                if k in x and x[k].shape == d[k].shape:
                    env_k = np.maximum(env_k, np.abs(d[k].astype(np.float64) - x[k].astype(np.float64)))
                d["env." + k] = env_k
        # per recorded step and link: 1 where the FMA or the x87 build's flow
        # class differs from this build's (the (link, step) pairs where the
        # reference itself flips a class; the parity test exempts the
        # class-selected coefficients only there)
        k = "s.link.flowClass"
        flip = np.zeros(d[k].shape, dtype=np.uint8)
        for b in (e, x):
            n = min(len(b[k]), len(d[k]))
            flip[:n] |= (b[k][:n] != d[k][:n]).astype(np.uint8)
        d["env.link.classFlip"] = flip
        d["env.x87.run.counts"] = x["run.counts"]
        d["env.x87.run.massbal"] = x["run.massbal"]
        for k in ("run.counts", "run.massbal"):
            d["env." + k] = e[k]
        with open(tmp + "_fma.rpt", "rb") as f, open(os.path.join(HERE, name + ".fma_rpt.txt"), "wb") as g:
            g.write(f.read())
        if name in X87_RPT:
            with open(tmp + "_x87.rpt", "rb") as f, open(os.path.join(HERE, name + ".x87_rpt.txt"), "wb") as g:
                g.write(f.read())
        with open(tmp + "_fma.out", "rb") as f:
            np.save(os.path.join(HERE, name + ".fma_out.npy"), np.frombuffer(f.read(), dtype=np.uint8))
    if name in ACTIONS:
        d["api.actions"] = np.frombuffer(ACTIONS[name].encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    with open(tmp + ".out", "rb") as f:
        out = f.read()
    np.save(os.path.join(HERE, name + ".ref_out.npy"), np.frombuffer(out, dtype=np.uint8))
    # the reference's report file (summary tables after swmm_report)
    with open(tmp + ".rpt", "rb") as f, open(os.path.join(HERE, name + ".ref_rpt.txt"), "wb") as g:
        g.write(f.read())
    saved = os.path.join(HERE, name + ".hsf")
    if os.path.exists(saved):
        os.replace(saved, os.path.join(HERE, name + ".ref.hsf"))
    print(name, len(d["s.dt"]), "steps", os.path.getsize(os.path.join(HERE, name + ".npz")), "bytes")


if __name__ == "__main__":
    for n in (sys.argv[1:] or CASES):
        make(n)
