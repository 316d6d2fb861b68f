import torch, time
dev = torch.device("cuda", 0)
torch.manual_seed(0)
x = torch.randn(4096, 768, device=dev, dtype=torch.float16)
w = torch.randn(3072, 768, device=dev, dtype=torch.float16) * 0.05
b = torch.randn(3072, device=dev, dtype=torch.float16) * 0.1
ref_lin = (x.float() @ w.float().t() + b.float())
exact = torch.nn.functional.gelu(ref_lin)
tanh = torch.nn.functional.gelu(ref_lin, approximate="tanh")
try:
    y = torch.ops.aten._addmm_activation(b, x, w.t(), use_gelu=True)
    print("addmm_activation dtype", y.dtype)
    print("max |y - gelu_erf|  =", (y.float() - exact).abs().max().item())
    print("max |y - gelu_tanh| =", (y.float() - tanh).abs().max().item())
    print("max |erf - tanh|    =", (exact - tanh).abs().max().item())
    # timing: fused vs linear + separate gelu
    xl = torch.randn(327680, 768, device=dev, dtype=torch.float16)
    for f, name in ((lambda: torch.ops.aten._addmm_activation(b, xl, w.t(), use_gelu=True), "fused"),
                    (lambda: torch.nn.functional.gelu(torch.nn.functional.linear(xl, w, b)), "separate")):
        for _ in range(3): f()
        torch.cuda.synchronize(); t = time.perf_counter()
        for _ in range(10): f()
        torch.cuda.synchronize(); print(name, (time.perf_counter() - t) / 10 * 1e3, "ms")
except Exception as e:
    print("error", e)
