"""Generates tests/golden/reference_config_development.json: the configuration the REFERENCE's
own loader produces from its own config files (load_config(env="development",
config_dir=/root/reference/configs), src/audio_rag/config/loader.py:119-173), dumped as data.

tests/test_reference_config.py builds this package's AudioRAG from that dump (written back out
as YAML), so the drop-in is checked against what a reference deployment actually loads, on the
GPU box too, where /root/reference does not exist.

Run in the build container:
    python tests/golden/make_config_fixture.py
"""

from __future__ import annotations

import json
import os
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import make_golden  # noqa: E402  (recording fakes for the engines the reference imports)


def main() -> None:
    for k in [k for k in os.environ if k.startswith("AUDIO_RAG__")]:
        del os.environ[k]  # the reference loader applies these; the fixture is the files alone
    make_golden.install_fakes()
    sys.path.insert(0, make_golden.REF_SRC)
    from audio_rag.config import load_config

    cfg = load_config(env="development", config_dir=make_golden.REF_CONFIGS)
    out = {
        "generator": "tests/golden/make_config_fixture.py (reference loader on reference configs)",
        "call": "load_config(env='development', config_dir='configs')",
        "config": json.loads(cfg.model_dump_json()),
    }
    path = HERE / "reference_config_development.json"
    path.write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print(f"wrote {path}")


if __name__ == "__main__":
    main()
