"""Synthetic-network generators (host logic, CPU)."""
import numpy as np

import netgen
import swmm5


def test_grid_counts_match_survey():
    assert netgen.grid_counts(224, 224) == (50177, 99905)
    assert netgen.grid_counts(707, 707) == (499850, 998285)
    assert netgen.grid_counts(1414, 1414) == (1999397, 3995965)


def test_grid_file_parses_with_expected_topology(tmp_path):
    p = tmp_path / "g.inp"
    nn, nl = netgen.write_grid(str(p), 7, 5)
    assert (nn, nl) == netgen.grid_counts(7, 5)
    s = swmm5.SWMM()
    assert s.open(str(p), str(tmp_path / "g.rpt"), str(tmp_path / "g.out")) == 0, s.getError()
    assert s.getCount(swmm5.NODE) == nn and s.getCount(swmm5.LINK) == nl
    # row-major numbering: +i link first, then +j link
    n1 = s.get_array("link.node1").astype(int)
    n2 = s.get_array("link.node2").astype(int)
    assert s.getName(swmm5.NODE, n1[0]) == "J0_0" and s.getName(swmm5.NODE, n2[0]) == "J1_0"
    assert s.getName(swmm5.NODE, n2[1]) == "J0_1"
    assert s.getName(swmm5.NODE, n2[-1]) == "OUT"
    slope = s.get_array("link.slope")
    assert np.all(slope > 0)
    s.close()


def test_example_has_reversed_conduit_and_offsets(tmp_path):
    p = tmp_path / "e.inp"
    netgen.write_example(str(p))
    s = swmm5.SWMM()
    assert s.open(str(p), str(tmp_path / "e.rpt"), str(tmp_path / "e.out")) == 0, s.getError()
    assert s.start_host() == 0
    direction = s.get_array("link.direction")
    off = s.get_array("link.offset1") + s.get_array("link.offset2")
    assert (direction < 0).any()           # adverse slope reversed under DW
    assert (off > 0).any()
    s.close()
