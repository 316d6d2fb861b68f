"""The drop-in at the configuration level: what a reference deployment loads from its own config
files (tests/golden/reference_config_development.json, produced by the reference's loader) must
validate here and select this package's MI355X store, with the reference's ingest behaviour as
the default (qdrant.py:183-220 sparse-drop)."""

import os
import sys
from pathlib import Path

import pytest
import yaml

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
import replay  # noqa: E402

REF_CONFIGS = Path("/root/reference/configs")


def test_reference_config_validates_and_selects_mi355x():
    from audio_rag_amd.config import AudioRAGConfig
    from audio_rag_amd.retrieval import MI355XRetriever, RetrievalRegistry

    cfg = AudioRAGConfig(**replay.reference_config())
    assert cfg.retrieval.backend == "qdrant"
    assert RetrievalRegistry.get(cfg.retrieval.backend) is MI355XRetriever
    assert RetrievalRegistry.get("mi355x") is MI355XRetriever
    # reference behaviour by default; keeping sparse vectors is an explicit opt-in
    assert cfg.retrieval.reproduce_sparse_drop is True
    assert cfg.retrieval.rrf_k == 2
    assert (cfg.retrieval.search_type, cfg.retrieval.top_k) == ("hybrid", 5)
    assert (cfg.reranking.top_k, cfg.reranking.initial_k) == (5, 20)


def test_rrf_k_must_be_positive():
    from pydantic import ValidationError

    from audio_rag_amd.config import RetrievalConfig

    with pytest.raises(ValidationError):
        RetrievalConfig(rrf_k=0)


def test_audiorag_from_reference_yaml(tmp_path):
    """AudioRAG.from_config on the reference's merged configuration written back as YAML: the
    lazy retriever wiring (orchestrator.py:48-57) builds the MI355X store under key "qdrant"."""
    from audio_rag_amd import AudioRAG
    from audio_rag_amd.retrieval import MI355XRetriever

    path = tmp_path / "reference.yaml"
    path.write_text(yaml.safe_dump(replay.reference_config()))
    rag = AudioRAG.from_config(config_path=path)

    class DimOnly:
        is_loaded = True
        dimension = 1024

    rag._embedder = DimOnly()
    assert isinstance(rag.retriever, MI355XRetriever)  # no device work at construction
    assert rag.retriever.config.collection_name == "audio_rag"


@pytest.mark.skipif(not REF_CONFIGS.is_dir(), reason="reference checkout not mounted")
def test_fixture_matches_reference_files():
    """This package's loader on the reference's own files gives the fixture's values."""
    from audio_rag_amd.config import load_config

    saved = {k: os.environ.pop(k) for k in list(os.environ) if k.startswith("AUDIO_RAG__")}
    try:
        cfg = load_config(env="development", config_dir=REF_CONFIGS)
    finally:
        os.environ.update(saved)
    want = replay.reference_config()
    got = cfg.model_dump()
    for section in ("retrieval", "embedding", "reranking"):
        for key, value in want[section].items():
            assert got[section][key] == value, (section, key)
    assert got["log_level"] == want["log_level"]
