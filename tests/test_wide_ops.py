"""CPU checks of the wide path's autograd helpers (ops/wide.py): the position-table gather whose
backward is a split-K one-hot GEMM, and the tall-skinny product with a split-K weight gradient, against
autograd's own gather / matmul gradients."""
import torch

from induction_network_on_fewrel_amd.ops.wide import SmallTableGather, TallSkinnyMM


def test_small_table_gather_backward_matches_index_backward():
    torch.manual_seed(0)
    for shape in ((301, 37), (64, 37), (5, 3)):   # token counts with / without split padding
        t = torch.randn(74, 5, requires_grad=True)
        idx = torch.randint(0, 74, shape)
        d = torch.randn(*shape, 5)
        out = SmallTableGather.apply(t, idx)
        assert torch.equal(out, t.detach()[idx])
        out.backward(d)
        t2 = t.detach().clone().requires_grad_(True)
        t2[idx].backward(d)
        torch.testing.assert_close(t.grad, t2.grad, rtol=1e-5, atol=1e-4)


def test_tall_skinny_mm_gradients():
    torch.manual_seed(1)
    for T in (8192, 100):   # split-K path and the single-GEMM fallback
        x = torch.randn(T, 500, requires_grad=True)
        w = torch.randn(500, 5, requires_grad=True)
        dy = torch.randn(T, 5)
        TallSkinnyMM.apply(x, w).backward(dy)
        x2 = x.detach().clone().requires_grad_(True)
        w2 = w.detach().clone().requires_grad_(True)
        (x2 @ w2).backward(dy)
        torch.testing.assert_close(x.grad, x2.grad)
        torch.testing.assert_close(w.grad, w2.grad, rtol=1e-4, atol=1e-3)


def test_word_table_cache_follows_identity_not_address():
    """word_table_bf16 must not hand a new table the rows of a freed one that sat at the same address
    (the caching allocator reuses addresses; a data_ptr key did exactly that), and must follow in-place
    updates (version counter)."""
    import gc
    from induction_network_on_fewrel_amd.ops.wide import word_table_bf16
    for i in range(4):
        a = torch.full((50, 8), float(i + 1))
        ta = word_table_bf16(a)
        assert torch.equal(ta.float(), a)
        del a, ta
        gc.collect()
        b = torch.full((50, 8), -float(i + 1))   # same shape, version 0, likely the same storage address
        assert torch.equal(word_table_bf16(b).float(), b)
        b.mul_(2.0)
        assert torch.equal(word_table_bf16(b).float(), b)
