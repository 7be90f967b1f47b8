"""ina.ragged_sort (csrc/kernels/ragged.hip) == the stable argsort plan it replaced (ops/encoder.py)."""
import pytest
import torch

from induction_network_on_fewrel_amd.ops import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("S,L", [(409600, 37), (1000, 37), (17, 64), (16 * 1025 + 3, 5), (1, 0), (1000000, 64)])
def test_ragged_sort_matches_stable_argsort(S, L):
    g = torch.Generator().manual_seed(S + L)
    NI = 5000
    lengths = torch.randint(0, L + 1, (NI,), generator=g, dtype=torch.int32).cuda()
    inst = torch.randint(0, NI, (S,), generator=g, dtype=torch.int32).cuda()
    inst_s, perm, tlen, slen = ops().ragged_sort(inst, lengths, L)
    lens = lengths.index_select(0, inst.long())
    ref_perm = torch.argsort(lens, stable=True)
    ref_slen = lens.index_select(0, ref_perm)
    ntiles = (S + 15) // 16
    last = torch.clamp(torch.arange(ntiles, device="cuda") * 16 + 15, max=S - 1)
    ref_tlen = torch.clamp(ref_slen.index_select(0, last), min=1)
    assert torch.equal(perm.long(), ref_perm)
    assert torch.equal(slen, ref_slen.int())
    assert torch.equal(inst_s, inst.index_select(0, ref_perm))
    assert torch.equal(tlen, ref_tlen.int())
