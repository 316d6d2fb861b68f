"""FFN block of the cross-encoder (up GEMM + bias, exact GELU, down GEMM + bias, add+LayerNorm)
over 1280 x 256 tokens: whole-batch vs token chunks small enough that the 3072-wide
intermediate stays in the 256 MB Infinity Cache between its producer and consumers."""
import sys
import torch
sys.path.insert(0, ".")
from audio_rag_amd._armi import call, ptr, stream_handle

dev = torch.device("cuda", 0)
M, d, ff = 1280 * 256, 768, 3072
g = torch.Generator(device=dev).manual_seed(0)
h1 = (torch.randn(M, d, device=dev, generator=g)).half()
wi = (torch.randn(ff, d, device=dev, generator=g) * 0.03).half()
bi = (torch.randn(ff, device=dev, generator=g) * 0.1).half()
wo = (torch.randn(d, ff, device=dev, generator=g) * 0.02).half()
bo = (torch.randn(d, device=dev, generator=g) * 0.1).half()
gam = torch.ones(d, device=dev)
bet = torch.zeros(d, device=dev)
lin = torch.nn.functional.linear
s = stream_handle()
out = torch.empty(M, d, dtype=torch.float16, device=dev)
res = torch.empty(M, d, dtype=torch.float16, device=dev)


def ffn(C):
    for c0 in range(0, M, C):
        c1 = min(M, c0 + C)
        x = h1[c0:c1]
        inter = lin(x, wi, bi)
        call("armi_enc_gelu_f16", ptr(inter), None, c1 - c0, ff, s)
        torch.addmm(bo, inter, wo.t(), out=out[c0:c1])
        call("armi_enc_add_layernorm_f16", ptr(out[c0:c1]), ptr(x), ptr(gam), ptr(bet), ptr(res[c0:c1]),
             c1 - c0, d, 1e-5, s)


ref = None
for rep in range(2):
    for C in (M, 65536, 32768, 16384, 8192):
        for _ in range(2):
            ffn(C)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            ffn(C)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        if C == M:
            ref = res.clone()
        same = torch.equal(res, ref)
        print(f"chunk {C:7d}: {ms:.3f} ms per FFN block  (identical to whole-batch: {same})")
