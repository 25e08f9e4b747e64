"""Cross-section cases of the geometry known-answer tests (test infrastructure).

Each case: (label, reference shape code (enums.h), the four [XSECTIONS]
parameters).  Codes: 1 CIRCULAR 2 FILLED_CIRCULAR 3 RECT_CLOSED 4 RECT_OPEN
5 TRAPEZOIDAL 6 TRIANGULAR 7 PARABOLIC 8 POWER 9 RECT_TRIANGULAR
10 RECT_ROUND 11 MODBASKETHANDLE 12 HORIZ_ELLIPSE 13 VERT_ELLIPSE 14 ARCH
15 EGG 16 HORSESHOE 17 GOTHIC 18 CATENARY 19 SEMIELLIPTICAL
20 BASKETHANDLE 21 SEMICIRCULAR 24 FORCE_MAIN.
"""
import numpy as np

SHAPES = [
    ("circular", 1, (1.5, 0, 0, 0)),
    ("filled_circular", 2, (3.0, 0.5, 0, 0)),
    ("rect_closed", 3, (3.0, 3.0, 0, 0)),
    ("rect_open", 4, (2.0, 3.0, 0, 0)),
    ("trapezoidal", 5, (2.0, 2.0, 1.5, 1.5)),
    ("triangular", 6, (2.0, 4.0, 0, 0)),
    ("parabolic", 7, (2.0, 4.0, 0, 0)),
    ("power", 8, (3.5, 4.0, 2.5, 0)),
    ("rect_triangular", 9, (4.0, 4.0, 1.0, 0)),
    ("rect_round", 10, (4.0, 4.0, 3.0, 0)),
    ("modbasket", 11, (3.0, 4.0, 2.5, 0)),
    ("modbasket_min_radius", 11, (3.0, 4.0, 1.0, 0)),
    ("horiz_ellipse", 12, (3.0, 4.5, 0, 0)),
    ("horiz_ellipse_code3", 12, (3, 0, 0, 0)),
    ("vert_ellipse", 13, (3.0, 2.0, 0, 0)),
    ("vert_ellipse_code2", 13, (2, 0, 0, 0)),
    ("arch_code5", 14, (5, 0, 0, 0)),
    ("arch_code60", 14, (60, 0, 0, 0)),
    ("arch", 14, (3.0, 4.0, 0, 0)),
    ("egg", 15, (1.5, 0, 0, 0)),
    ("horseshoe", 16, (1.5, 0, 0, 0)),
    ("gothic", 17, (2.0, 0, 0, 0)),
    ("catenary", 18, (2.0, 0, 0, 0)),
    ("semielliptical", 19, (2.0, 0, 0, 0)),
    ("baskethandle", 20, (2.5, 0, 0, 0)),
    ("semicircular", 21, (2.0, 0, 0, 0)),
    ("force_main", 24, (1.0, 120, 0, 0)),
]
FUNCS = ["AofY", "WofY", "RofY", "YofA", "RofA", "SofA", "AofS", "dSdA", "Ycrit"]


def points(fn, par):
    """Evaluation points of relation fn (1-based FUNCS index) for a section."""
    u = np.concatenate([np.linspace(0.0, 1.0, 41), [1e-7, 1e-4, 0.003, 0.0399, 0.04, 0.5 + 1e-9, 0.97,
                                                    0.985, 0.999, 1.0 - 1e-12]])
    if fn in (1, 2, 3):
        return u * par["yFull"]
    if fn in (4, 5, 6, 8):
        return u * par["aFull"]
    if fn == 7:
        return np.concatenate([u, [1.01, 1.05, 1.2]]) * par["sFull"]
    # critical depth: flows up to about the full-pipe critical flow
    qc = par["aFull"] * np.sqrt(32.2 * par["aFull"] / max(par["wMax"], 1e-6))
    return np.concatenate([u, [1.5, 3.0]]) * qc
