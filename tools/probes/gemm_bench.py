"""armi_enc_linear_f16 (hand-written gfx950 GEMM, fused bias / bias +
exact GELU) against torch's hipBLASLt linear (+ the standalone armi GELU pass) on the
cross-encoder's four GEMM shapes at configs[2]'s token count (1280 pairs x 256 tokens). Prints
one JSON line per shape."""
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from audio_rag_amd._armi import call, ptr, stream_handle  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


def main():
    dev = torch.device("cuda", 0)
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 327680
    g = torch.Generator(device=dev).manual_seed(0)
    for name, n, k, epi in (("qkv", 2304, 768, 0), ("wo", 768, 768, 0), ("ffn_up", 3072, 768, 1),
                            ("ffn_down", 768, 3072, 0)):
        if os.environ.get("GEMM_SHAPES") and name not in os.environ["GEMM_SHAPES"].split(","):
            continue
        x = torch.randn((M, k), generator=g, device=dev).half()
        w = (torch.randn((n, k), generator=g, device=dev) / k ** 0.5).half()
        b = torch.randn(n, generator=g, device=dev) * 0.1
        bh = b.half()
        out = torch.empty((M, n), dtype=torch.float16, device=dev)
        s = stream_handle()

        def armi():
            call("armi_enc_linear_f16", ptr(x), ptr(w), ptr(b), ptr(out), M, n, k, epi, s)

        def lt():
            y = torch.nn.functional.linear(x, w, bh)
            if epi:
                call("armi_enc_gelu_f16", ptr(y), None, M, n, s)
            return y


        ta = timeit(armi)
        tl = timeit(lt) if not os.environ.get("GEMM_NO_LT") else float("nan")
        flops = 2.0 * M * n * k
        # correctness on a slice (first and last tokens)
        errs = []
        for sl in (slice(0, 512), slice(M - 300, M)):
            ref = x[sl].float() @ w.float().t() + b
            if epi:
                ref = torch.nn.functional.gelu(ref)
            errs.append((out[sl].float() - ref).abs().max().item())
        print(json.dumps({"shape": name, "m": M, "n": n, "k": k, "epilogue": ["bias", "bias+gelu"][epi],
                          "armi_ms": ta, "armi_tflops": flops / ta / 1e9,
                          "hipblaslt_ms": tl, "hipblaslt_tflops": flops / tl / 1e9,
                          "max_abs_err_vs_fp32": max(errs)}), flush=True)
        del x, w, out


if __name__ == "__main__":
    main()
