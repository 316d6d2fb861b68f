import logging

from audio_rag_amd.utils.decorators import require_loaded, timed


def get_logger(name: str) -> logging.Logger:
    return logging.getLogger(name)


def setup_logging(level: str = "INFO") -> None:
    logging.basicConfig(level=getattr(logging, level, logging.INFO),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")


__all__ = ["timed", "require_loaded", "get_logger", "setup_logging"]
