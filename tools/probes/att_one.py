"""armi_enc_attention_f16 at the configs[2] rerank shape (1280 pairs x L 256, 12 heads x 64),
launched 10 times: the program profiled by tools/probes/att_pmc.sh."""
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
for _ in range(10):
    assert lib.armi_enc_attention_f16(qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(), n, L, H, dh,
                                      dh ** -0.5, s) == 0
torch.cuda.synchronize()
