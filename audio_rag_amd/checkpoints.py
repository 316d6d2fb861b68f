"""Local checkpoints and tokenizers for the two encoders of the query path.

The reference loads its models by name: BGEM3FlagModel(config.model) (embeddings/bge.py:47-55)
and CrossEncoder(config.model, max_length=512) (reranking/bge.py:50-55), both resolving a Hugging
Face hub id or a local directory. This module does the same offline:

  * config.model names a local directory, or a hub id whose snapshot is already in the local
    Hugging Face cache (huggingface_hub, local_files_only: nothing is ever fetched);
  * weights load through weights-only loaders only: model.safetensors via safetensors, or a
    pytorch_model.bin via torch.load(weights_only=True); BGE-M3's sparse head sparse_linear.pt
    the same way;
  * tokenizer.json loads through the `tokenizers` library (the fast XLM-R tokenizer the
    reference's sentencepiece model converts to).

When config.model resolves to nothing on disk the encoders keep their seeded stand-in weights
and the stand-in tokenizer (audio_rag_amd.text), and say so in the log.
"""

from __future__ import annotations

import logging
import os
from pathlib import Path

import torch

from audio_rag_amd.text import BOS, EOS, PAD, UNK

logger = logging.getLogger(__name__)


def resolve_local(name: str | None) -> Path | None:
    """A directory holding config.json for `name` (a path, or a cached hub snapshot), else None."""
    if not name:
        return None
    p = Path(os.path.expanduser(name))
    if p.is_dir():
        return p if (p / "config.json").exists() else None
    try:
        from huggingface_hub import snapshot_download

        snap = Path(snapshot_download(name, local_files_only=True))
        return snap if (snap / "config.json").exists() else None
    except Exception:
        return None


def state_dict(path: Path) -> dict[str, torch.Tensor] | None:
    """The checkpoint's tensors through a weights-only loader (None without a weights file)."""
    st = path / "model.safetensors"
    if st.exists():
        from safetensors.torch import load_file

        return load_file(str(st))
    pt = path / "pytorch_model.bin"
    if pt.exists():
        return torch.load(str(pt), map_location="cpu", weights_only=True)
    return None


def load_pretrained(cls, path: Path, **kwargs):
    """cls(config.json) with the checkpoint's tensors (weights-only, above). Keys are matched with
    or without the model's base prefix ("roberta."), as from_pretrained does; a missing tensor
    raises, an unused pooler / buffer is ignored."""
    from transformers import AutoConfig

    sd = state_dict(path)
    if sd is None:
        raise FileNotFoundError(f"{path}: no model.safetensors or pytorch_model.bin")
    cfg = AutoConfig.from_pretrained(str(path), local_files_only=True)
    model = cls(cfg, **kwargs)
    want = model.state_dict()
    pre = getattr(model, "base_model_prefix", "") + "."
    fixed = {}
    for k, v in sd.items():
        if k not in want:
            if pre + k in want:
                k = pre + k
            elif k.startswith(pre) and k[len(pre):] in want:
                k = k[len(pre):]
        if k in want:
            fixed[k] = v
    missing = [k for k in want if k not in fixed and not k.endswith("position_ids")]
    if missing:
        raise ValueError(f"{path}: checkpoint lacks {len(missing)} tensors, e.g. {missing[:3]}")
    model.load_state_dict(fixed, strict=False)
    model.eval()
    return model


class HFTokenizer:
    """tokenizer.json through `tokenizers`, with the interface of text.HashTokenizer: ids without
    special tokens (tokenize), and <s> ids </s> truncated to max_length (encode)."""

    def __init__(self, path: Path):
        from tokenizers import Tokenizer

        self.tok = Tokenizer.from_file(str(path))
        self.tok.no_truncation()
        self.tok.no_padding()
        tid = self.tok.token_to_id
        self.bos = tid("<s>") if tid("<s>") is not None else BOS
        self.eos = tid("</s>") if tid("</s>") is not None else EOS
        self.pad = tid("<pad>") if tid("<pad>") is not None else PAD
        self.unk = tid("<unk>") if tid("<unk>") is not None else UNK
        self.vocab_size = self.tok.get_vocab_size()
        if (self.bos, self.pad, self.eos) != (BOS, PAD, EOS):
            raise ValueError(f"{path}: special ids {(self.bos, self.pad, self.eos)} differ from "
                             f"XLM-R's (<s>, <pad>, </s>) = {(BOS, PAD, EOS)}")

    @property
    def special_ids(self) -> frozenset:
        return frozenset((self.bos, self.pad, self.eos, self.unk))

    def tokenize(self, text: str) -> list[int]:
        return list(self.tok.encode(text, add_special_tokens=False).ids)

    def encode(self, text: str, max_length: int = 8192) -> list[int]:
        ids = self.tokenize(text)[: max(max_length - 2, 0)]
        return [self.bos, *ids, self.eos]


def load_tokenizer(path: Path | None):
    """HFTokenizer for a checkpoint directory holding tokenizer.json, else None."""
    if path is None or not (path / "tokenizer.json").exists():
        return None
    return HFTokenizer(path / "tokenizer.json")


def tokenizer_for(name: str | None):
    """The tokenizer of the checkpoint `name` resolves to on disk, else None (no checkpoint: the
    encoders keep their seeded stand-ins and the stand-in tokenizer). A checkpoint whose weights
    are on disk without tokenizer.json raises: its load() would run the real weights on the
    stand-in tokenizer's ids and return wrong vectors without any error."""
    path = resolve_local(name)
    tok = load_tokenizer(path)
    if tok is None and path is not None and (
            (path / "model.safetensors").exists() or (path / "pytorch_model.bin").exists()):
        raise FileNotFoundError(f"{path}: checkpoint weights without tokenizer.json (convert the "
                                "sentencepiece model to tokenizer.json next to the weights)")
    return tok
