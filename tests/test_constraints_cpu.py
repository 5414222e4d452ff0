"""CPU: the reference-format constraint parsers (`solver/solver.py:396-476`, `:603-663`) and the no-fallback rule."""
import pytest
import torch

import fem355  # noqa: F401
from fem355 import _capi, constraints as CS

SPC = [{"node": 10, "dofs": [0, 1, 2], "value": 0.0}, {"node": 20, "dofs": [0], "value": 0.01}]
RBE2 = [{"master": 15, "slaves": [21, 22, 23], "dofs": [0, 1, 2]}, {"master": 50, "slaves": [51, 52], "dofs": [0, 2]}]
RBE3 = [{"master": 15, "slaves": [21, 22, 23], "dofs": [0, 1, 2], "weights": [1.0, 2.0, 1.0]},
        {"master": 50, "slaves": [51, 52], "dofs": [2, 0], "weights": [1.0, 3.0]}]


def test_parse_spc_and_rbe2_order_and_dtypes():
    n, d, v = CS.parse_spc_list(SPC, device="cpu")
    assert n.dtype == d.dtype == torch.int32 and v.dtype == torch.float64
    assert n.tolist() == [10, 10, 10, 20] and d.tolist() == [0, 1, 2, 0] and v.tolist() == [0.0, 0.0, 0.0, 0.01]
    s, m, d = CS.parse_rbe2_list(RBE2, device="cpu")
    assert s.tolist() == [21, 21, 21, 22, 22, 22, 23, 23, 23, 51, 51, 52, 52]
    assert m.tolist() == [15] * 9 + [50] * 4 and d.tolist() == [0, 1, 2] * 3 + [0, 2, 0, 2]
    assert all(t.dtype == torch.int32 for t in (s, m, d))
    e = CS.parse_spc_list([], device="cpu")
    assert all(t.numel() == 0 for t in e)


def test_parse_rbe3_offsets_and_weight_sums():
    m, s, d, w, inds, sums = CS.parse_rbe3_list(RBE3, device="cpu")
    assert inds.dtype == torch.int64 and inds.tolist() == [0, 9, 13]
    assert sums.tolist() == [4.0, 4.0]
    assert s[9:].tolist() == [51, 51, 52, 52] and d[9:].tolist() == [2, 0, 2, 0] and w[9:].tolist() == [1, 1, 3, 3]
    assert m.tolist() == [15] * 9 + [50] * 4


def test_apply_loads_in_place_in_order():
    F = torch.zeros((4, 3), dtype=torch.float32)
    CS.apply_loads_to_F(F, [{"node": 1, "force": [1.0, 2.0, 3.0]}, {"node": 1, "force": [0.5, 0.0, -3.0]}])
    assert F[1].tolist() == [1.5, 2.0, 0.0] and float(F.abs().sum()) == 3.5


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device path")
def test_constraint_set_has_no_cpu_fallback():
    with pytest.raises(_capi.FemError):
        CS.ConstraintSet(100, 3, "cpu", CS.parse_spc_list(SPC, "cpu"), CS.parse_rbe2_list(RBE2, "cpu"))
    with pytest.raises(_capi.FemError):
        CS.enforce_constraints(torch.zeros(100, 3, dtype=torch.float64), torch.zeros(100, 3, dtype=torch.float64),
                               *CS.parse_spc_list(SPC, "cpu"), *CS.parse_rbe2_list(RBE2, "cpu"))
