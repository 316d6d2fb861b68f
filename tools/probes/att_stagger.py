"""armi_enc_attention_f16 at 1280 x 256 (configs[2]) under phase-stagger settings
(ARMI_ATT_STAGGER cycles, ARMI_ATT_STAGGER_MODE), alternating, same process."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from audio_rag_amd import _armi  # noqa: E402

lib = _armi.load()
dev = torch.device("cuda", 0)
n, L, H, dh = 1280, 256, 12, 64
g = torch.Generator(device=dev).manual_seed(0)
qkv = (torch.randn(n * L, 3 * H * dh, device=dev, generator=g) * 0.5).half()
mask = torch.ones(n, L, dtype=torch.int32, device=dev)
ctx = torch.empty(n * L, H * dh, dtype=torch.float16, device=dev)
s = torch.cuda.current_stream().cuda_stream
f = lambda: lib.armi_enc_attention_f16(qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(), n, L, H, dh, dh ** -0.5, s)
settings = [(0, 0), (12000, 0), (6000, 0), (20000, 0), (12000, 1), (6000, 1), (20000, 1)]
ref = None
for rep in range(3):
    for cyc, mode in settings:
        os.environ["ARMI_ATT_STAGGER"] = str(cyc)
        os.environ["ARMI_ATT_STAGGER_MODE"] = str(mode)
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        if ref is None:
            ref = ctx.clone()
        same = torch.equal(ctx, ref)
        print(f"stagger {cyc:6d} mode {mode}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us  identical {same}", flush=True)
