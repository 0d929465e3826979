"""The C-ABI library loads and exports every symbol include/gwa.h declares; without a GPU every
compute entry point fails loudly (no silent CPU fallback)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(REPO, "include", "gwa.h")).read()
    return sorted(set(re.findall(r"\b(gwa_[a-z_]+)\s*\(", txt)))


def test_header_and_python_mirror_agree():
    import gwa
    assert sorted(gwa.EXPORTS) == _declared()


def test_library_exports_every_declared_symbol():
    import gwa
    L = gwa.lib()
    for sym in _declared():
        assert hasattr(L, sym), sym


def test_config_defaults_match_reference():
    import gwa
    c = gwa._Config()
    gwa.lib().gwa_config_default(ctypes.byref(c))
    # A/AlignmentScoreConfig.java:37-77, A/AlignmentConfig.java:61-72
    assert abs(c.k - 0.1) < 1e-7 and c.strategy == 0 and c.report_type == 0 and c.top_l == 5
    assert (c.num_gap_open, c.num_gap_ext, c.num_split) == (1, 4, 1)
    assert (c.match, c.mismatch, c.gap_open, c.gap_ext, c.split_open) == (1, 3, 11, 4, 11)
    assert (c.indel_end_skip, c.band_width) == (5, 31)
    d = gwa.AlignmentConfig()._c()
    for f in ("k", "strategy", "report_type", "top_l", "num_split", "band_width"):
        assert getattr(c, f) == getattr(d, f)


def test_max_edit_distance_float_semantics():
    import gwa
    c = gwa.AlignmentConfig()
    assert c.getMaximumEditDistance(100) == 10
    assert c.getMaximumEditDistance(8) == 0      # BWAlignTest.align3: floor(8 * 0.1f) = 0
    assert c.getMaximumEditDistance(150) == 15
    c.k = 2
    assert c.getMaximumEditDistance(100) == 2


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="GPU present")
def test_no_gpu_fails_loudly():
    import gwa
    with pytest.raises(gwa.GwaError, match="no HIP device|device"):
        gwa.FMIndexOnGenome.buildFromSequence("seq", "AAGCCTAGTTTCCTTG")
