import pytest
import torch

pytestmark = pytest.mark.gpu


def test_mfma_lane_maps(C):
    g = torch.Generator().manual_seed(0)
    A = torch.randn(16, 32, generator=g)
    B = torch.randn(32, 16, generator=g)  # asymmetric B catches a transposed C-write
    Dbf, Df = C.mfma_selftest(A.cuda(), B.cuda())
    ref_bf = A.bfloat16().float() @ B.bfloat16().float()
    torch.testing.assert_close(Dbf.cpu(), ref_bf, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(Df.cpu(), A @ B, rtol=1e-5, atol=1e-5)
