"""Drop-in check: the reference's own command-line driver, unmodified.

oracle/Makefile (target runswmm_dropin) compiles the reference's
src/run/main.c -- which only includes swmm5.h and calls swmm_getVersion,
swmm_run, swmm_getError and swmm_getWarnings -- against this repository's
include/swmm5.h and links it to libswmm5_mi355x.so.  Running that binary on a
golden input must produce a binary results file with the reference's exact
layout and values (same tolerance as test_gpu_parity.py), i.e. a reference
caller switches engines by relinking, with no source change.

The binary is built in this container (where /root/reference exists) and
travels to the GPU box with the rest of oracle/_ref/.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

import _golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "oracle", "_ref", "runswmm_dropin")


def _need_cli():
    if not os.path.exists(CLI):
        pytest.skip("oracle/_ref/runswmm_dropin not built (needs /root/reference at build time)")


def test_dropin_cli_links_engine():
    """The reference driver resolves every swmm_* symbol from our library."""
    _need_cli()
    out = subprocess.run(["ldd", CLI], capture_output=True, text=True).stdout
    assert "libswmm5_mi355x.so" in out and "not found" not in out


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["example", "grid12_var_qual"])
def test_dropin_cli_matches_reference(name, tmp_path):
    _need_cli()
    rpt, out = str(tmp_path / "x.rpt"), str(tmp_path / "x.out")
    r = subprocess.run([CLI, _golden.inp(name), rpt, out], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "There are errors" not in r.stdout, r.stdout
    mine = open(out, "rb").read()
    ref = _golden.ref_out(name)
    assert len(mine) == len(ref)
    start = struct.unpack("<i", ref[-16:-12])[0]
    assert mine[:start] == ref[:start]
    assert mine[-24:] == ref[-24:]
    a = np.frombuffer(mine[start:-24], dtype="<f4")
    b = np.frombuffer(ref[start:-24], dtype="<f4")
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    assert "Flow Routing Continuity" in open(rpt).read()
