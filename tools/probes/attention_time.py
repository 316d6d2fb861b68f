"""Times armi_enc_attention_f16 at the rerank bench shape (1280 pairs x L 256, 12 heads x 64)
and reports the achieved HBM rate of its algorithmic bytes (QKV read once + ctx written).
Optional extra argv: paths of other builds of libarmi.so to time alternately (A/B)."""
import ctypes
import sys
import torch
sys.path.insert(0, ".")
from audio_rag_amd import _armi

libs = [("current", _armi.load())]
for p in sys.argv[1:]:
    lib = ctypes.CDLL(p)
    fn = lib.armi_enc_attention_f16
    fn.restype, fn.argtypes = _armi.SIGNATURES["armi_enc_attention_f16"]
    libs.append((p.rsplit("/", 1)[-1], lib))

dev = torch.device("cuda", 0)
for n, L in ((1280, 256), (64, 512), (20, 96)):
    H, dh = 12, 64
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = (torch.randn(n * L, 3 * H * dh, device=dev, generator=g) * 0.5).half()
    mask = torch.ones(n, L, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    outs = []
    for rep in range(2):
        for name, lib in libs:
            ctx = torch.empty(n * L, H * dh, dtype=torch.float16, device=dev)
            f = lambda: lib.armi_enc_attention_f16(qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(), n, L, H, dh,
                                                   dh ** -0.5, s)
            for _ in range(3):
                assert f() == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            it = 20
            e0.record()
            for _ in range(it):
                f()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / it
            byts = qkv.numel() * 2 + ctx.numel() * 2
            fl = 4.0 * n * H * L * L * dh
            print(f"{name:16s} n={n} L={L}: {ms*1e3:.1f} us  {byts/ms/1e9:.2f} TB/s  {fl/ms/1e9:.1f} TFLOP/s")
            if rep == 0:
                outs.append(ctx)
    for o in outs[1:]:
        print("  identical to current:", torch.equal(o, outs[0]))
