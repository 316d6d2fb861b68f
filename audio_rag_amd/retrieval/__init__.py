"""Retrieval backends (mirrors src/audio_rag/retrieval/__init__.py)."""
