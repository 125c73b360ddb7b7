"""Numerics of the large-tile MFMA GEMM (csrc/gemm.hip) against fp32 PyTorch: C = A B^T with the
plain / bias epilogue, and the GPT-2 MLP backward epilogue dZ = (dY W2) * gelu'(z + b) with its
bias-gradient column sums. Shapes cover ragged M (rows past M load as zeros and are not stored),
a single K-tile and long K."""
import pytest
import torch

from determined_clone_amd.ops import _ext

pytestmark = pytest.mark.gpu


def _C():
    C = _ext.load()
    assert C.__file__.endswith("_C.so")
    return C


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 512, 128), (1000, 768, 768), (4096, 1024, 1024),
                                   (333, 3072, 1024), (2048, 1024, 4096)])
@pytest.mark.parametrize("bias", [False, True])
def test_gemm_nt_matches_fp32(M, N, K, bias):
    C = _C()
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
    # asymmetric bias so a transposed or shifted epilogue shows
    bb = torch.linspace(-1, 1, N, device="cuda") if bias else None
    c = C.gemm_nt(a, b, bb)
    ref = a.float() @ b.float().t() + (bb if bias else 0)
    assert c.shape == (M, N) and c.dtype == torch.bfloat16
    assert _rel(c, ref) < 8e-3
    # every row / column written (no stale tile): max error bounded everywhere
    assert (c.float() - ref).abs().max().item() < 0.1 * ref.abs().max().item()


def test_gemm_nt_batched_rows_and_identity():
    """[B, S, K] activations; A = I picks B's rows exactly (a transposed C-write fails this)."""
    C = _C()
    torch.manual_seed(1)
    N, K = 512, 256
    b = torch.randn(N, K, device="cuda").bfloat16()
    eye = torch.eye(K, device="cuda").bfloat16().reshape(2, K // 2, K)
    c = C.gemm_nt(eye, b)
    assert c.shape == (2, K // 2, N)
    torch.testing.assert_close(c.reshape(K, N).float(), b.float().t()[:K], rtol=0, atol=0)


@pytest.mark.parametrize("T_,E,F", [(333, 768, 3072), (8192, 1024, 4096), (96, 256, 512)])
def test_gemm_nt_dgelu(T_, E, F):
    C = _C()
    torch.manual_seed(0)
    dy = torch.randn(T_, E, device="cuda").bfloat16()
    w2 = (torch.randn(E, F, device="cuda") * E ** -0.5).bfloat16()
    z = torch.randn(T_, F, device="cuda").bfloat16()
    bias = torch.randn(F, device="cuda") * 0.5
    dz, partial = C.gemm_nt_dgelu(dy, w2.t().contiguous(), z, bias)
    zr = (z.float() + bias).requires_grad_(True)
    torch.nn.functional.gelu(zr, approximate="tanh").backward(dy.float() @ w2.float())
    assert dz.shape == (T_, F)
    assert _rel(dz, zr.grad) < 1e-2
    assert partial.shape == ((T_ + 255) // 256, F)
    assert _rel(partial.sum(0), zr.grad.sum(0)) < 1e-2
