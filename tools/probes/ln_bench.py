import sys, torch
sys.path.insert(0, '.')
from audio_rag_amd._armi import call, ptr, stream_handle
dev = torch.device('cuda', 0)
M, W = 327680, 768
x = torch.randn(M, W, device=dev).half(); r = torch.randn(M, W, device=dev).half()
g = torch.randn(W, device=dev); b = torch.randn(W, device=dev)
o = torch.empty(M, W, dtype=torch.float16, device=dev)
s = stream_handle()
f = lambda: call('armi_enc_add_layernorm_f16', ptr(x), ptr(r), ptr(g), ptr(b), ptr(o), M, W, 1e-5, s)
for _ in range(5): f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50): f()
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 50
print('add_layernorm_f16', M, W, round(ms * 1e3, 1), 'us', round(3 * M * W * 2 / ms / 1e9, 0), 'GB/s')
