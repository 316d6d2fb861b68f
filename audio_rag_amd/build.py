"""Builds libarmi.so (HIP kernels + C ABI, gfx950) in-tree with hipcc.

The library is a plain shared object with an extern "C" surface (include/armi.h); Python loads
it with ctypes (audio_rag_amd/_armi.py). It is written to audio_rag_amd/_lib/ so the GPU box
receives it with the repository snapshot.
"""

from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OUT_DIR = PKG / "_lib"
# ARMI_LIB_OUT: write a probe build (ARMI_BUILD_FLAGS variants) elsewhere; load it with ARMI_LIB_PATH
LIB = Path(os.environ["ARMI_LIB_OUT"]) if os.environ.get("ARMI_LIB_OUT") else OUT_DIR / "libarmi.so"
OBJ_DIR = ROOT / "build" / "armi_obj"

SOURCES = ["armi_common.cpp", "index.hip", "dense.hip", "sparse.hip", "rrf.hip", "encoder.hip",
           "attention.hip", "gemm.hip", "stream.cpp"]
ARCH = os.environ.get("ARMI_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-ffp-contract=off",
         f"-I{ROOT / 'include'}"]
# extra flags for diagnostic builds, e.g. ARMI_BUILD_FLAGS=-DARMI_SPARSE_PROFILE
FLAGS += os.environ.get("ARMI_BUILD_FLAGS", "").split()


def _digest(path: Path, headers: list[Path]) -> str:
    h = hashlib.sha256()
    for p in [path, *headers]:
        h.update(p.read_bytes())
    h.update(" ".join(FLAGS + [ARCH]).encode())
    return h.hexdigest()[:16]


def _compile(src: str, headers: list[Path], source_digest: str) -> Path:
    path = CSRC / src
    extra = []
    tag = _digest(path, headers)
    if src == "armi_common.cpp":  # carries armi_source_digest(): rebuilt whenever any source changes
        extra = [f'-DARMI_SOURCE_DIGEST="{source_digest}"']
        tag = hashlib.sha256((tag + source_digest).encode()).hexdigest()[:16]
    obj = OBJ_DIR / f"{path.stem}-{tag}.o"
    if obj.exists():
        return obj
    cmd = [HIPCC, *FLAGS, *extra, "-c", str(path), "-o", str(obj)]
    if src.endswith(".hip"):
        cmd.insert(1, f"--offload-arch={ARCH}")
    else:
        cmd += ["-x", "c++"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{res.stdout}\n{res.stderr}")
    return obj


def build(verbose: bool = False) -> Path:
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    LIB.parent.mkdir(parents=True, exist_ok=True)
    headers = sorted(CSRC.glob("*.h")) + [ROOT / "include" / "armi.h"]
    from audio_rag_amd._armi import source_digest

    sd = source_digest()
    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(lambda s: _compile(s, headers, sd), SOURCES))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs),
           "-Wl,-rpath,/opt/rocm/lib", "-Wl,-z,defs", "-lamdhip64", "-lpthread"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed:\n{res.stdout}\n{res.stderr}")
    os.replace(tmp, LIB)
    keep = {o.name for o in objs}
    for stale in OBJ_DIR.glob("*.o"):  # objects of superseded sources
        if stale.name not in keep and not os.environ.get("ARMI_LIB_OUT"):
            stale.unlink()
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build(verbose="-q" not in sys.argv)
