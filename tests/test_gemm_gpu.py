"""Own gfx950 bf16 GEMM (csrc/kernels/gemm.hip, ina.bert_gemm) vs a plain PyTorch fp32 GEMM of the same
bf16 inputs: plain / bias, bias + GELU with the pre-activation aux, and GELU' * C with the bias-gradient
column-sum slab.  Shapes include the BERT-base FFN (K = 768 / 3072, N = 768 / 3072) and ragged M tails."""
import pytest
import torch

from induction_network_on_fewrel_amd.models import bert as B

pytestmark = pytest.mark.gpu
dev = torch.device("cuda")


def _ops():
    from induction_network_on_fewrel_amd.ops._ext import ops
    return ops()


def _close(a, b, rtol):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err / scale < rtol, f"max err {err} vs scale {scale}"


def _gelu_grad(u):
    return 0.5 * (1.0 + torch.erf(u * 0.7071067811865476)) + u * 0.3989422804014327 * torch.exp(-0.5 * u * u)


SHAPES = [(256, 256, 64), (300, 512, 192), (1000, 768, 768), (4133, 3072, 768), (2048 + 37, 768, 3072), (97, 256, 128),
          (8292, 3072, 768), (17000, 1024, 192)]   # the last two: more tiles than CUs (persistent blocks), odd K-step count


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("bias", [False, True])
def test_gemm_plain(M, N, K, bias):
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=dev) if bias else None
    y, _ = _ops().bert_gemm(x, w, b, None, 0)
    ref = x.float() @ w.float().t()
    if bias:
        ref = ref + b
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    _close(y, ref, 1e-2)


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_bias_gelu(M, N, K):
    torch.manual_seed(1 + M)
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=dev) * 0.5
    y, aux = _ops().bert_gemm(x, w, b, None, 1)
    pre = x.float() @ w.float().t() + b
    _close(aux, pre, 1e-2)
    _close(y, B.gelu(pre), 1e-2)


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_dgelu_slab(M, N, K):
    torch.manual_seed(2 + M)
    dy = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
    aux = (torch.randn(M, N, device=dev) * 2).bfloat16()
    d, slab = _ops().bert_gemm(dy, w, None, aux, 2)
    ref = (dy.float() @ w.float().t()) * _gelu_grad(aux.float())
    _close(d, ref, 1e-2)
    assert slab.shape == (2 * ((M + 255) // 256), N)
    _close(slab.sum(0), ref.sum(0), 1e-2)


def test_gemm_deterministic():
    torch.manual_seed(5)
    M, N, K = 1500, 3072, 768
    dy = torch.randn(M, K, device=dev).bfloat16()
    w = torch.randn(N, K, device=dev).bfloat16()
    aux = torch.randn(M, N, device=dev).bfloat16()
    a1, s1 = _ops().bert_gemm(dy, w, None, aux, 2)
    a2, s2 = _ops().bert_gemm(dy, w, None, aux, 2)
    assert torch.equal(a1, a2) and torch.equal(s1, s2)


def test_gemm_rejects_bad_shapes():
    x = torch.randn(64, 100, device=dev).bfloat16()
    w = torch.randn(256, 100, device=dev).bfloat16()
    with pytest.raises(RuntimeError):
        _ops().bert_gemm(x, w, None, None, 0)   # K % 64 != 0
    x = torch.randn(64, 128, device=dev).bfloat16()
    w = torch.randn(204, 128, device=dev).bfloat16()
    with pytest.raises(RuntimeError):
        _ops().bert_gemm(x, w, None, None, 0)   # N % 8 != 0
    with pytest.raises(RuntimeError):
        _ops().gemm_nn(x, torch.randn(128, 204, device=dev).bfloat16(), None, None, 0)   # N % 8 != 0
    with pytest.raises(RuntimeError):
        _ops().gemm_wgrad(torch.randn(64, 36, device=dev).bfloat16(), torch.randn(64, 64, device=dev).bfloat16(), 0)


@pytest.mark.parametrize("M,N,K", [(300, 264, 128), (4133, 2312, 768), (97, 8, 64)])
def test_gemm_nt_ragged_n(M, N, K):
    """NT with N not a multiple of 256 (rows of B past N clamped on load, never stored)."""
    torch.manual_seed(N + K)
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=dev)
    y, _ = _ops().bert_gemm(x, w, b, None, 0)
    _close(y, x.float() @ w.float().t() + b, 1e-2)


NN_SHAPES = [(256, 256, 64), (300, 768, 768), (4133, 768, 3072), (2048 + 37, 3072, 768), (97, 264, 128),
             (17000, 768, 2304), (1000, 1032, 192)]   # (M, N, K): ragged M / N tails, more tiles than CUs


@pytest.mark.parametrize("M,N,K", NN_SHAPES)
@pytest.mark.parametrize("epi", [0, 2, 4])
def test_gemm_nn(M, N, K, epi):
    """NN layout (dgrad dx = dy W with W [K][N] read K-major through ds_read_b64_tr_b16): plain, GELU' * C with
    the bias-gradient column sums (the FFN-down dgrad without a transposed weight copy), and the residual
    epilogue (C added in place into res) -- vs the fp32 product of the same bf16 inputs."""
    torch.manual_seed(M + N + K + epi)
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(K, N, device=dev) / K ** 0.5).bfloat16()
    ref = a.float() @ w.float()
    if epi == 0:
        y, _ = _ops().gemm_nn(a, w, None, None, 0)
        _close(y, ref, 1e-2)
    elif epi == 2:
        aux = (torch.randn(M, N, device=dev) * 2).bfloat16()
        d, slab = _ops().gemm_nn(a, w, aux, None, 2)
        r = ref * _gelu_grad(aux.float())
        _close(d, r, 1e-2)
        assert slab.shape == (2 * ((M + 255) // 256), N)
        _close(slab.sum(0), r.sum(0), 1e-2)
    else:
        res = torch.randn(M, N, device=dev).bfloat16()
        r = ref + res.float()
        y, _ = _ops().gemm_nn(a, w, None, res, 4)
        assert y.data_ptr() == res.data_ptr()
        _close(y, r, 1e-2)


WG_SHAPES = [(4096, 768, 768, 0), (6400, 2304, 768, 0), (1000, 256, 512, 3), (8192, 576, 1024, 0), (6216, 40, 264, 0),
             (102400 // 8, 3072, 768, 0), (64, 8, 8, 1), (5000, 768, 3072, 7)]   # (K, M, N, splits)


@pytest.mark.parametrize("K,M,N,splits", WG_SHAPES)
def test_gemm_wgrad(K, M, N, splits):
    """TN split-K weight-gradient GEMM: sum of the fp32 slabs = a^T b over all K (ragged K: K-major rows past K
    read zeros; ragged M / N tiles; explicit and automatic split counts) vs fp32 torch."""
    torch.manual_seed(K + M + N)
    a = torch.randn(K, M, device=dev).bfloat16()
    b = torch.randn(K, N, device=dev).bfloat16()
    slab = _ops().gemm_wgrad(a, b, splits)
    torch.cuda.synchronize()
    assert slab.shape[1:] == (M, N) and slab.dtype == torch.float32
    if splits > 0:
        assert slab.shape[0] == splits
    ref = a.float().t() @ b.float()
    err = (slab.sum(0) - ref).abs()
    assert (err / (ref.abs() + K ** 0.5)).max().item() < 1e-4, err.max().item()


def test_gemm_wgrad_strided_and_deterministic():
    """Operands that are column slices of wider rows (the paper configuration's [x | h] rows), bitwise repeatable."""
    torch.manual_seed(11)
    big = torch.randn(3000, 640, device=dev).bfloat16()
    b = torch.randn(3000, 520, device=dev).bfloat16()
    a = big[:, 64:640]
    s1 = _ops().gemm_wgrad(a, b[:, :512], 0)
    s2 = _ops().gemm_wgrad(a, b[:, :512], 0)
    assert torch.equal(s1, s2)
    ref = a.float().t() @ b[:, :512].float()
    err = (s1.sum(0) - ref).abs()
    assert (err / (ref.abs() + 3000 ** 0.5)).max().item() < 1e-4


@pytest.mark.parametrize("K,MI,NJ,splits", [(64, 40, 4000, 0), (40960, 40, 4000, 0), (1280, 64, 1000, 3), (640, 16, 8, 0),
                                            (4096, 48, 2056, 7), (192, 8, 264, 5)])
def test_gemm_tn_slab(K, MI, NJ, splits):
    """Reduction GEMM (csrc/kernels/gemm_tn.hip): slab[s] summed = A[:, :MI]^T B over all K, vs fp32 torch.
    Includes the headline dM shape (K = 8192 episodes x 5 classes, MI = H = 40, NJ = h H = 4000), column tails
    past the last 256-wide tile, more splits than K-steps per split divides, and an A wider than MI."""
    torch.manual_seed(K + MI + NJ)
    lda = MI + (8 if MI < 64 else 0)
    A = torch.randn(K, lda, device=dev).bfloat16()
    Bm = torch.randn(K, NJ, device=dev).bfloat16()
    slab = _ops().gemm_tn_slab(A, Bm, MI, splits)
    torch.cuda.synchronize()
    ref = A[:, :MI].float().t() @ Bm.float()
    got = slab.sum(0)
    assert slab.shape[1:] == (MI, NJ)
    err = (got - ref).abs()
    # fp32 accumulation of exact bf16 products: only summation-order differences
    assert (err / (ref.abs() + (K ** 0.5))).max().item() < 1e-4, err.max().item()

