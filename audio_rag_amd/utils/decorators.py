"""@timed and @require_loaded (src/audio_rag/utils/decorators.py:14-23, 75-86)."""

import functools
import logging
import time

logger = logging.getLogger("audio_rag_amd.utils.decorators")


def timed(func):
    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        start = time.perf_counter()
        result = func(*args, **kwargs)
        elapsed = time.perf_counter() - start
        logger.info(f"{func.__qualname__} completed in {elapsed:.2f}s")
        return result

    return wrapper


def require_loaded(func):
    @functools.wraps(func)
    def wrapper(self, *args, **kwargs):
        if not self.is_loaded:
            logger.info(f"{self.__class__.__name__}: Auto-loading model")
            self.load()
        return func(self, *args, **kwargs)

    return wrapper
