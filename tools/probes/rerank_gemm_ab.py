"""Cross-encoder forward at configs[2]'s shape (1,280 pairs x 256 tokens, bge-reranker-base,
fp16) with the linear layers on each GEMM implementation of CrossEncoderXLMR (class attribute
gemm_impl): "mixed" (hipBLASLt + armi_enc_linear_f16 for FFN-up) and "armi" (armi_enc_linear_f16
for all four). Prints one JSON line per form: forward
ms (graph replay), TFLOP/s and the max score difference against the first form."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from audio_rag_amd.reranking.xlmr import CrossEncoderXLMR, build_reranker  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, L = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (1280, 256)))
    forms = sys.argv[3].split(",") if len(sys.argv) > 3 else ["mixed", "armi"]
    enc = CrossEncoderXLMR(build_reranker(5), dev)
    enc.to_dtype(torch.float16)
    g = torch.Generator(device=dev).manual_seed(1)
    ids = torch.randint(4, 250000, (n, L), generator=g, device=dev, dtype=torch.int32)
    ids[:, 0] = 0
    ids[:, 17] = 2
    ids[:, 18] = 2
    ids[:, -1] = 2
    mask = torch.ones_like(ids)
    first = None
    for form in forms:
        enc.gemm_impl = form
        enc.__dict__.pop("_graphs", None)  # recapture with this form's kernels
        for _ in range(2):
            p = enc.forward(ids, mask)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        it = 5
        for _ in range(it):
            p = enc.forward(ids, mask)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / it
        if first is None:
            first = p
        print(json.dumps({"form": form, "n": n, "L": L, "forward_ms": ms,
                          "tflops": enc.flops(n, L) / ms / 1e9,
                          "max_abs_diff_vs_first": (p - first).abs().max().item()}), flush=True)


if __name__ == "__main__":
    main()
