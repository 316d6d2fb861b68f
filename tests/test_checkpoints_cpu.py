"""Local checkpoints for the two encoders (audio_rag_amd/checkpoints.py), on the CPU: weights-only
loading of model.safetensors / pytorch_model.bin (with and without the "roberta." prefix),
BGE-M3's sparse_linear.pt, tokenizer.json through `tokenizers`, and the seeded stand-in when
config.model names nothing on disk. Reference: BGEM3FlagModel(config.model)
(embeddings/bge.py:47-55), CrossEncoder(config.model) (reranking/bge.py:50-55)."""

import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
from ckpt_util import WORDS, save_bge_m3, save_reranker, write_tokenizer  # noqa: E402

TINY = dict(vocab_size=len(WORDS) + 4, hidden_size=64, num_hidden_layers=2,
            num_attention_heads=4, intermediate_size=128, max_position_embeddings=64)


def _same(a, b):
    sa, sb = a.state_dict(), b.state_dict()
    assert sa.keys() == sb.keys()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


def test_bge_m3_dir_loads_weights_sparse_head_and_tokenizer(tmp_path):
    from audio_rag_amd.checkpoints import HFTokenizer
    from audio_rag_amd.embeddings.bge_m3 import build_bge_m3, load_bge_m3

    save_bge_m3(tmp_path / "m3", 7, TINY)
    model, sparse, tok = load_bge_m3(str(tmp_path / "m3"), seed=99)
    ref_model, ref_sparse = build_bge_m3(7, TINY)
    _same(model, ref_model)
    _same(sparse, ref_sparse)
    assert isinstance(tok, HFTokenizer)
    assert tok.encode("the lecture zebra") == [0, 4, 6, 3, 2]  # zebra: <unk>
    assert tok.tokenize("gradient descent") == [7, 8]
    assert tok.special_ids == frozenset((0, 1, 2, 3))


def test_pytorch_bin_and_prefixed_keys(tmp_path):
    """A pytorch_model.bin (weights_only torch.load) whose keys carry the base-model prefix, and
    a classification checkpoint: both match from_pretrained's key handling."""
    from transformers import XLMRobertaModel

    from audio_rag_amd.checkpoints import load_pretrained
    from audio_rag_amd.embeddings.bge_m3 import build_bge_m3
    from audio_rag_amd.reranking.bge import load_reranker
    from audio_rag_amd.reranking.xlmr import build_reranker

    ref, _ = build_bge_m3(3, TINY)
    d = tmp_path / "bin"
    d.mkdir()
    ref.config.save_pretrained(str(d))
    torch.save({"roberta." + k: v for k, v in ref.state_dict().items()}, str(d / "pytorch_model.bin"))
    _same(load_pretrained(XLMRobertaModel, d, add_pooling_layer=False), ref)
    save_reranker(tmp_path / "rr", 11, TINY)
    hf, tok = load_reranker(str(tmp_path / "rr"), seed=0)
    _same(hf, build_reranker(11, TINY))
    assert tok is not None and tok.tokenize("model data") == [11, 12]


def test_absent_model_keeps_seeded_stand_in(tmp_path):
    from audio_rag_amd.checkpoints import resolve_local
    from audio_rag_amd.embeddings.bge_m3 import build_bge_m3, load_bge_m3

    assert resolve_local("BAAI/bge-m3-not-cached-here") is None
    assert resolve_local(str(tmp_path)) is None  # a directory without config.json
    model, _, tok = load_bge_m3("BAAI/bge-m3-not-cached-here", seed=5, arch=TINY)
    _same(model, build_bge_m3(5, TINY)[0])
    assert tok is None


def test_checkpoint_missing_tensor_raises(tmp_path):
    import pytest
    from safetensors.torch import save_file
    from transformers import XLMRobertaModel

    from audio_rag_amd.checkpoints import load_pretrained
    from audio_rag_amd.embeddings.bge_m3 import build_bge_m3

    ref, _ = build_bge_m3(3, TINY)
    ref.config.save_pretrained(str(tmp_path))
    sd = {k: v.contiguous() for k, v in ref.state_dict().items() if "layer.1." not in k}
    save_file(sd, str(tmp_path / "model.safetensors"))
    write_tokenizer(tmp_path)
    with pytest.raises(ValueError, match="lacks"):
        load_pretrained(XLMRobertaModel, tmp_path, add_pooling_layer=False)
