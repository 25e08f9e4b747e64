"""Known-answer tests of the cross-section relations (xsect.c) against vectors
the reference itself produced (tests/golden/xsect_kat.npz, made by
tests/golden/make_xsect_kat.py from the reference build).

Host evaluation (the code that builds the kernels' constants) must be
bit-identical; the device evaluation runs the kernels' own xsect.h code with
the GPU's libm and must agree within the north_star tolerance."""
import numpy as np
import pytest

import _golden  # noqa: F401  (puts the package on sys.path)
import swmm5
from _xsect_cases import SHAPES, FUNCS

KAT = np.load(_golden.GOLDEN + "/xsect_kat.npz", allow_pickle=False)
IDS = [s[0] for s in SHAPES]


@pytest.mark.parametrize("k", range(len(SHAPES)), ids=IDS)
def test_section_parameters_bit_identical(k):
    _, code, p = SHAPES[k]
    np.testing.assert_array_equal(swmm5.xsect(code, p, 0), KAT["params_%d" % k])


@pytest.mark.parametrize("k", range(len(SHAPES)), ids=IDS)
def test_host_relations_bit_identical(k):
    _, code, p = SHAPES[k]
    for fi, fname in enumerate(FUNCS, start=1):
        x, y = KAT["x_%d_%d" % (k, fi)], KAT["y_%d_%d" % (k, fi)]
        np.testing.assert_array_equal(swmm5.xsect(code, p, fi, x), y, err_msg=fname)


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(SHAPES)), ids=IDS)
def test_device_relations_match_reference(k):
    _, code, p = SHAPES[k]
    for fi, fname in enumerate(FUNCS, start=1):
        x, y = KAT["x_%d_%d" % (k, fi)], KAT["y_%d_%d" % (k, fi)]
        np.testing.assert_allclose(swmm5.xsect(code, p, fi, x, device=True), y, rtol=1e-9, atol=1e-12,
                                   err_msg=fname)
