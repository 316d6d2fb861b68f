"""Helpers of the checkpoint tests: a WordLevel tokenizer.json with XLM-R's special ids and
sequence layout (<s> A </s> / <s> A </s></s> B </s>), written with the `tokenizers` library, and
seeded encoders saved with save_pretrained (model.safetensors + config.json)."""

from pathlib import Path

WORDS = ("the of lecture gradient descent loss function model data training step rate "
         "speaker minute question answer vector search chunk audio transcript learning "
         "neural network layer weight bias batch epoch optimizer memory cache kernel").split()


def write_tokenizer(path: Path) -> dict:
    from tokenizers import Tokenizer, models, pre_tokenizers, processors

    vocab = {"<s>": 0, "<pad>": 1, "</s>": 2, "<unk>": 3}
    for w in WORDS:
        vocab.setdefault(w, len(vocab))
    tok = Tokenizer(models.WordLevel(vocab, unk_token="<unk>"))
    tok.pre_tokenizer = pre_tokenizers.Whitespace()
    tok.post_processor = processors.TemplateProcessing(
        single="<s> $A </s>", pair="<s> $A </s> </s> $B </s>",
        special_tokens=[("<s>", 0), ("</s>", 2)])
    tok.save(str(path / "tokenizer.json"))
    return vocab


def save_bge_m3(path: Path, seed: int, arch: dict) -> None:
    import torch

    from audio_rag_amd.embeddings.bge_m3 import build_bge_m3

    model, sparse = build_bge_m3(seed, arch)
    path.mkdir(parents=True, exist_ok=True)
    model.save_pretrained(str(path))
    torch.save(sparse.state_dict(), str(path / "sparse_linear.pt"))
    write_tokenizer(path)


def save_reranker(path: Path, seed: int, arch: dict) -> None:
    from audio_rag_amd.reranking.xlmr import build_reranker

    path.mkdir(parents=True, exist_ok=True)
    build_reranker(seed, arch).save_pretrained(str(path))
    write_tokenizer(path)
