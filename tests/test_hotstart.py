"""Hot start files (hotstart.c) against the reference.

CPU: reading a hot start file written by the reference gives the reference's
post-swmm_start state bit for bit (covered for every golden case by
test_host_init; here the error paths).  GPU: the file the engine saves at
swmm_end matches the reference's file for the same run -- same header and
record layout, float32 values within rtol 1e-6 (the north_star tolerance;
values near 0 within 1e-6 absolute) -- and a run resumed from the engine's
own file matches the run resumed from the reference's (rtol 1e-5 after 720
steps: the two files' float32 states may differ in the last ulp).

A truncated file is ERROR 335 here; the reference's readFloat ignores the
short read and keeps the previous value (hotstart.c:500-518).
"""
import os
import shutil
import struct

import numpy as np
import pytest

import _golden
import swmm5

HDR = 15 + 6 * 4


def _copy_case(name, tmp_path, hsf_name=None):
    shutil.copy(os.path.join(_golden.GOLDEN, name + ".inp"), tmp_path)
    ref = os.path.join(_golden.GOLDEN, "example_hotsave.ref.hsf")
    shutil.copy(ref, tmp_path / (hsf_name or "example_hotsave.ref.hsf"))
    return str(tmp_path / (name + ".inp"))


def _start_host(inp, tmp_path):
    s = swmm5.SWMM()
    assert s.open(inp, str(tmp_path / "h.rpt"), str(tmp_path / "h.out")) == 0, s.getError()
    return s, s.start_host()


def test_missing_hot_start_file_is_error_331(tmp_path):
    inp = _copy_case("example_hot", tmp_path)
    os.remove(tmp_path / "example_hotsave.ref.hsf")
    s, rc = _start_host(inp, tmp_path)
    assert rc == 331
    s.close()


def test_incompatible_hot_start_file_is_error_333(tmp_path):
    inp = _copy_case("example_hot", tmp_path)
    p = tmp_path / "example_hotsave.ref.hsf"
    b = bytearray(p.read_bytes())
    struct.pack_into("<i", b, 15 + 2 * 4, 999)          # node count
    p.write_bytes(bytes(b))
    s, rc = _start_host(inp, tmp_path)
    assert rc == 333
    s.close()


def test_truncated_hot_start_file_is_error_335(tmp_path):
    inp = _copy_case("example_hot", tmp_path)
    p = tmp_path / "example_hotsave.ref.hsf"
    p.write_bytes(p.read_bytes()[:HDR + 40])
    s, rc = _start_host(inp, tmp_path)
    assert rc == 335
    s.close()


def test_reference_file_layout():
    b = open(os.path.join(_golden.GOLDEN, "example_hotsave.ref.hsf"), "rb").read()
    assert b[:15] == b"SWMM5-HOTSTART4"
    nsub, nland, nn, nl, P, units = struct.unpack_from("<6i", b, 15)
    d = _golden.load("example_hotsave")
    assert (nsub, nland) == (0, 0)
    assert (nn, nl, P) == tuple(int(x) for x in d["counts"][:3])
    assert len(b) == HDR + 4 * (nn * (2 + P) + nl * (3 + P))


def _run_to_end(inp, tmp_path):
    s = swmm5.SWMM()
    assert s.open(inp, str(tmp_path / "g.rpt"), str(tmp_path / "g.out")) == 0, s.getError()
    assert s.start(True) == 0, s.getError()
    while True:
        err, t = s.step()
        assert err == 0, s.getError()
        if t == 0.0:
            break
    assert s.end() == 0, s.getError()
    s.close()


@pytest.mark.gpu
def test_saved_hot_start_matches_reference(tmp_path):
    inp = _golden.inp("example_hotsave")
    _run_to_end(inp, tmp_path)
    mine = open(os.path.join(os.path.dirname(inp), "example_hotsave.hsf"), "rb").read()
    ref = open(os.path.join(_golden.GOLDEN, "example_hotsave.ref.hsf"), "rb").read()
    assert len(mine) == len(ref)
    assert mine[:HDR] == ref[:HDR]
    a = np.frombuffer(mine[HDR:], dtype="<f4")
    b = np.frombuffer(ref[HDR:], dtype="<f4")
    np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_resume_from_engine_file_matches_resume_from_reference_file(tmp_path):
    save_dir = tmp_path / "save"
    save_dir.mkdir()
    shutil.copy(os.path.join(_golden.GOLDEN, "example_hotsave.inp"), save_dir)
    _run_to_end(str(save_dir / "example_hotsave.inp"), save_dir)
    # resume from the engine's file, compare against the golden resumed run
    run_dir = tmp_path / "run"
    run_dir.mkdir()
    shutil.copy(os.path.join(_golden.GOLDEN, "example_hot.inp"), run_dir)
    shutil.copy(save_dir / "example_hotsave.hsf", run_dir / "example_hotsave.ref.hsf")
    d = _golden.load("example_hot")
    s = swmm5.SWMM()
    assert s.open(str(run_dir / "example_hot.inp"), str(run_dir / "r.rpt"), str(run_dir / "r.out")) == 0
    assert s.start(False) == 0, s.getError()
    n = 0
    while True:
        err, t = s.step()
        assert err == 0, s.getError()
        n += 1
        if t == 0.0:
            break
    depth = s.get_array("node.newDepth")
    flow = s.get_array("link.newFlow")
    np.testing.assert_allclose(depth, d["s.node.newDepth"][-1], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(flow, d["s.link.newFlow"][-1], rtol=1e-5, atol=1e-6)
    s.end()
    s.close()
