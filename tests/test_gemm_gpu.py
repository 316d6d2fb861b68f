"""armi_enc_linear_f16 (the hand-written gfx950 GEMM of the cross-encoder's linear layers, fused
bias / bias + exact-erf GELU epilogues; include/armi.h) against a torch fp32 reference of the same
op: out = x . w^T + b (nn.Linear, XLMRobertaLayer as CrossEncoder.predict runs it,
src/audio_rag/reranking/bge.py:119-123), GELU(out) for the intermediate dense. fp16 operands,
fp32 accumulate, fp16 output: tolerance = fp16 output rounding (2^-10 relative) + 1e-3 absolute.
Shapes cover full and partial 256-token blocks, every XLM-R base width and a K of 3072, with
asymmetric operands (a transposed or mis-ordered output fails)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m,n,k,epi", [(256, 256, 128, 0), (1000, 768, 768, 0),
                                       (2048, 3072, 768, 1), (517, 768, 3072, 0),
                                       (300, 2304, 768, 0), (4096, 768, 768, 1),
                                       (77, 512, 192, 1),
                                       # several tiles per workgroup: the K-tile stream crosses
                                       # tile boundaries (next tile staged during an epilogue)
                                       (70001, 2304, 768, 0), (20000, 3072, 768, 1),
                                       (9000, 768, 3072, 0)])
def test_linear_f16_matches_fp32(gpu, m, n, k, epi):
    from audio_rag_amd._armi import call, ptr, stream_handle

    g = torch.Generator(device=gpu).manual_seed(m + n + k)
    x = torch.randn((m, k), generator=g, device=gpu).half()
    w = (torch.randn((n, k), generator=g, device=gpu) / k ** 0.5).half()
    w[:, 0] += torch.arange(n, device=gpu).half() * 1e-3  # asymmetric in (feature, k)
    b = torch.randn(n, generator=g, device=gpu) * 0.1
    out = torch.full((m, n), float("nan"), dtype=torch.float16, device=gpu)
    call("armi_enc_linear_f16", ptr(x), ptr(w), ptr(b), ptr(out), m, n, k, epi, stream_handle())
    torch.cuda.synchronize()
    ref = x.float() @ w.float().t() + b
    if epi:
        ref = torch.nn.functional.gelu(ref)  # exact erf GELU
    assert not torch.isnan(out).any()
    torch.testing.assert_close(out.float(), ref, rtol=2 ** -10, atol=1e-3)


def test_linear_f16_rejects_bad_shapes(gpu):
    from audio_rag_amd._armi import ArmiError, call, stream_handle

    with pytest.raises(ArmiError):
        call("armi_enc_linear_f16", None, None, None, None, 10, 100, 768, 0, stream_handle())
    with pytest.raises(ArmiError):
        call("armi_enc_linear_f16", None, None, None, None, 10, 256, 100, 0, stream_handle())


@pytest.mark.parametrize("m,n,k,epi", [(1, 3072, 1024, 0), (7, 1024, 1024, 0), (16, 4096, 1024, 1),
                                       (17, 1024, 4096, 0), (32, 3072, 1024, 1),
                                       (12, 16, 256, 0),
                                       # XLM-R base widths: the 8-wave k = 768 and the 16-wave
                                       # k = 3072 instances, both epilogues
                                       (1, 2304, 768, 0), (17, 3072, 768, 1), (32, 768, 768, 0),
                                       (1, 768, 3072, 0), (17, 768, 3072, 1), (32, 768, 3072, 0),
                                       # row blocks (the batched query encode): m > 32
                                       (33, 1024, 1024, 1), (100, 3072, 1024, 0),
                                       (257, 1024, 4096, 0), (70, 16, 1024, 0)])
def test_linear_small_m_matches_fp32(gpu, m, n, k, epi):
    """armi_enc_linear_small_f16 (the query encodes' weight-stream GEMM) against the same torch
    fp32 reference; rows of the output buffer past m stay untouched."""
    from audio_rag_amd._armi import call, ptr, stream_handle

    g = torch.Generator(device=gpu).manual_seed(7 * m + n + k)
    x = torch.randn((m, k), generator=g, device=gpu).half()
    w = (torch.randn((n, k), generator=g, device=gpu) / k ** 0.5).half()
    w[:, 0] += torch.arange(n, device=gpu).half() * 1e-3
    b = torch.randn(n, generator=g, device=gpu) * 0.1
    out = torch.full((m + 2, n), float("nan"), dtype=torch.float16, device=gpu)
    call("armi_enc_linear_small_f16", ptr(x), ptr(w), ptr(b), ptr(out), m, n, k, epi,
         stream_handle())
    torch.cuda.synchronize()
    ref = x.float() @ w.float().t() + b
    if epi:
        ref = torch.nn.functional.gelu(ref)
    assert not torch.isnan(out[:m]).any()
    assert torch.isnan(out[m:]).all()
    torch.testing.assert_close(out[:m].float(), ref, rtol=2 ** -10, atol=1e-3)


def test_linear_small_m_rows_independent(gpu):
    """A row's output does not depend on m or on the other rows (the batched query encode's
    premise): row r of an m-row call equals the 1-row call on x[r], bit for bit, for every k
    instance."""
    from audio_rag_amd._armi import call, ptr, stream_handle

    for k, n in ((1024, 3072), (4096, 1024), (768, 2304), (3072, 768)):
        g = torch.Generator(device=gpu).manual_seed(k)
        x = torch.randn((75, k), generator=g, device=gpu).half()
        w = (torch.randn((n, k), generator=g, device=gpu) / k ** 0.5).half()
        b = torch.randn(n, generator=g, device=gpu) * 0.1
        full = torch.empty((75, n), dtype=torch.float16, device=gpu)
        call("armi_enc_linear_small_f16", ptr(x), ptr(w), ptr(b), ptr(full), 75, n, k, 1,
             stream_handle())
        for r in (0, 31, 32, 50, 74):
            one = torch.empty((1, n), dtype=torch.float16, device=gpu)
            xr = x[r:r + 1].contiguous()
            call("armi_enc_linear_small_f16", ptr(xr), ptr(w), ptr(b), ptr(one), 1, n, k, 1,
                 stream_handle())
            torch.cuda.synchronize()
            assert torch.equal(one[0], full[r]), (k, r)

