"""ctypes binding of libarmi.so (the C ABI declared in include/armi.h).

This is the only way the package reaches the GPU: there is no CPU or PyTorch fallback for the
retrieval kernels. If the library is missing or fails to load, every caller gets
``ArmiUnavailable`` immediately (build it with ``python -m audio_rag_amd.build`` or
``__graft_entry__.build()``).
"""

from __future__ import annotations

import ctypes
import hashlib
import os
import threading
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "_lib" / "libarmi.so"
CSRC = Path(__file__).resolve().parent / "csrc"
HEADER = Path(__file__).resolve().parents[1] / "include" / "armi.h"

ARMI_OK = 0
ARMI_FLAG_CERTIFIED = 1
ARMI_FLAG_FALLBACK = 2
ARMI_FLAG_FILTERED = 4
TIMING_DENSE_SCAN, TIMING_SPARSE_SCAN, TIMING_ENCODER_GEMM, TIMING_SPARSE_STAGE = 0, 1, 2, 3
SCAN_FP16, SCAN_INT8_FILTER, SCAN_TILED_FP16, SCAN_TILED_INT8 = 0, 1, 2, 3  # armi_dense_scan_form
ABI_VERSION = 2

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int32 = ctypes.c_int32
c_int64 = ctypes.c_int64
c_size_t = ctypes.c_size_t
c_float = ctypes.c_float

# name -> (restype, argtypes); mirrors include/armi.h exactly
SIGNATURES: dict[str, tuple] = {
    "armi_last_error": (ctypes.c_char_p, []),
    "armi_abi_version": (c_int, []),
    "armi_source_digest": (ctypes.c_char_p, []),
    "armi_index_create": (c_int, [c_int, c_void_p, c_int64, c_int, c_int64, ctypes.POINTER(c_void_p), c_void_p]),
    "armi_dense_scan_form": (c_int, [c_void_p, c_int, c_int]),
    "armi_dense_scan_nontemporal": (c_int, [c_void_p, c_int, c_int]),
    "armi_index_destroy": (c_int, [c_void_p]),
    "armi_index_rows": (c_int64, [c_void_p]),
    "armi_index_dim": (c_int, [c_void_p]),
    "armi_index_invalid_rows": (c_int64, [c_void_p]),
    "armi_index_norms": (c_int, [c_void_p, ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p)]),
    "armi_dense_workspace_bytes": (c_size_t, [c_void_p, c_int, c_int]),
    "armi_dense_topk": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "armi_dense_exact_workspace_bytes": (c_size_t, [c_void_p, c_int, c_int]),
    "armi_dense_exact_topk": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "armi_topk_merge_shards": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                       c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "armi_topk_merge_shards_packed": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64,
                                              c_int64, c_int, c_int, c_int, c_int, c_void_p,
                                              c_void_p, c_void_p, c_void_p, c_void_p]),
    "armi_query_slots_pack": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                      c_void_p, c_void_p]),
    "armi_query_slots_unpack": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int64, c_int, c_int,
                                        c_void_p, c_void_p, c_void_p, c_void_p]),
    "armi_scan_timing_enable": (c_int, [c_int]),
    "armi_scan_timing_read": (c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_int64)]),
    "armi_kernel_timing_read": (c_int, [c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_int64)]),
    "armi_stream_create": (c_int, [c_void_p, c_int, c_int, ctypes.c_double, ctypes.POINTER(c_void_p)]),
    "armi_stream_create_hybrid": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.c_double,
                                          ctypes.POINTER(c_void_p)]),
    "armi_stream_destroy": (c_int, [c_void_p]),
    "armi_stream_stop": (c_int, [c_void_p]),
    "armi_stream_submit": (c_int, [c_void_p, c_void_p, ctypes.POINTER(c_int64)]),
    "armi_stream_submit_hybrid": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                          ctypes.POINTER(c_int64)]),
    "armi_stream_submit_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                      c_void_p, ctypes.POINTER(c_int64)]),
    "armi_stream_wait": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                 ctypes.c_double]),
    "armi_stream_stats": (c_int, [c_void_p, ctypes.POINTER(c_int64), ctypes.POINTER(c_int64)]),
    "armi_stream_loadgen": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                    ctypes.c_double, ctypes.c_uint64, c_void_p,
                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_int64),
                                    c_void_p, c_void_p]),
    "armi_sparse_index_create": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int32,
                                         c_int64, ctypes.POINTER(c_void_p), c_void_p]),
    "armi_sparse_index_destroy": (c_int, [c_void_p]),
    "armi_sparse_workspace_bytes": (c_size_t, [c_void_p, c_int, c_int]),
    "armi_sparse_index_set_filter": (c_int, [c_void_p, c_int, c_void_p]),
    "armi_sparse_topk": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "armi_rrf_fuse": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                              c_void_p, c_void_p, c_void_p, c_void_p]),
    "armi_enc_layernorm_residual": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                            c_int, c_float, c_void_p]),
    "armi_enc_masked_softmax": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p]),
    "armi_enc_bias_gelu": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "armi_enc_embed": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p]),
    "armi_enc_embed_f16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
                                   c_void_p]),
    "armi_enc_cls_head_sigmoid": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_int, c_int, c_int, c_void_p]),
    "armi_enc_attention_f16": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                       c_float, c_void_p]),
    "armi_enc_attention_cls_f16": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                           c_float, c_void_p]),
    "armi_enc_layernorm_residual_f16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                c_void_p, c_int64, c_int, c_float, c_void_p]),
    "armi_enc_gelu_f16": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "armi_enc_linear_f16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int,
                                    c_int, c_void_p]),
    "armi_enc_linear_small_f16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                          c_int, c_int, c_void_p]),
    "armi_enc_add_layernorm_f16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                           c_int, c_float, c_void_p]),
}


def source_digest() -> str | None:
    """sha256 (16 hex digits) over the library's sources: every csrc/*.hip, *.cpp, *.h and
    include/armi.h, by name and content. build.py compiles it into libarmi.so
    (armi_source_digest), and load() refuses a library built from other sources. None when the
    sources are not present next to the package."""
    if not CSRC.is_dir() or not HEADER.exists():
        return None
    h = hashlib.sha256()
    files = sorted(p for p in CSRC.iterdir() if p.suffix in (".hip", ".cpp", ".h"))
    for f in [*files, HEADER]:
        h.update(f.name.encode() + b"\0" + f.read_bytes() + b"\0")
    return h.hexdigest()[:16]


class ArmiUnavailable(RuntimeError):
    """libarmi.so is missing or unloadable: the MI355X path cannot run."""


class ArmiError(RuntimeError):
    """A libarmi call returned a non-zero status."""

    def __init__(self, fn: str, code: int, message: str):
        super().__init__(f"{fn} failed (status {code}): {message}")
        self.fn = fn
        self.code = code


_lock = threading.Lock()
_lib: ctypes.CDLL | None = None


def load(path: str | os.PathLike | None = None) -> ctypes.CDLL:
    """Loads libarmi.so once. torch is imported first so that the library binds to the same
    HIP runtime instance (libamdhip64.so.7) that owns torch's device allocations."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  (binds the process to torch's HIP runtime first)

        # ARMI_LIB_PATH: another build of the library (A/B measurements of two builds)
        p = Path(path or os.environ.get("ARMI_LIB_PATH") or LIB_PATH)
        if not p.exists():
            raise ArmiUnavailable(
                f"{p} not found: build it with `python -m audio_rag_amd.build` (hipcc, gfx950)")
        try:
            lib = ctypes.CDLL(str(p))
        except OSError as e:
            raise ArmiUnavailable(f"cannot load {p}: {e}") from e
        for name, (restype, argtypes) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = restype
            fn.argtypes = argtypes
        if lib.armi_abi_version() != ABI_VERSION:
            raise ArmiUnavailable(f"{p}: ABI version {lib.armi_abi_version()} != {ABI_VERSION}")
        want = source_digest()
        got = lib.armi_source_digest().decode()
        # ARMI_AB_OTHER_SOURCES=1 (with ARMI_LIB_PATH only): time a build of other sources, e.g.
        # the previous commit's kernel, beside this tree's on one box (A/B probes; never the
        # in-tree library, which always has to match csrc/)
        ab = bool(os.environ.get("ARMI_LIB_PATH")) and os.environ.get("ARMI_AB_OTHER_SOURCES") == "1"
        if want is not None and got != want and not ab:
            raise ArmiUnavailable(f"{p} was built from other sources (digest {got}, csrc/ is "
                                  f"{want}): rebuild it with `python -m audio_rag_amd.build`")
        _lib = lib
        return lib


def call(name: str, *args) -> int:
    """Calls an int-status entry point and raises ArmiError on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != ARMI_OK:
        msg = lib.armi_last_error().decode(errors="replace")
        raise ArmiError(name, rc, msg)
    return rc


def query(name: str, *args):
    """Calls a non-status entry point (sizes, counters) and returns its value."""
    return getattr(load(), name)(*args)


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(stream=None) -> int:
    """hipStream_t of a torch.cuda.Stream (default: the current stream)."""
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
