"""CPU: host-side argument checks of the Python binding (no GPU calls)."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))


def test_colmajor_view_checks():
    """crt_finish's C check: a column-major sub-matrix view with ld > rows is accepted; a view whose
    storage ends before the last column, a transposed (row-major) view and ld < rows are rejected"""
    import gemmul8 as G
    big = torch.zeros((12, 20), dtype=torch.float64)
    G._check_colmajor("C", big[1:11, :15], 15, 10, 20)   # 10 columns of 15 rows, ld 20
    G._check_colmajor("C", big, 20, 12, 20)              # the whole buffer
    G._check_colmajor("C", big.view(-1), 15, 12, 20)     # a flat buffer
    with pytest.raises(ValueError, match="storage"):
        G._check_colmajor("C", big[3:12, :15], 15, 10, 20)
    with pytest.raises(ValueError, match="column-major"):
        G._check_colmajor("C", big[:, :15].t(), 15, 10, 20)
    with pytest.raises(ValueError, match="leading dimension"):
        G._check_colmajor("C", big, 21, 12, 20)
