"""YAML + environment configuration loader.

Same merge order and environment syntax as src/audio_rag/config/loader.py:119-173:
schema defaults < base.yaml < {env}.yaml < explicit file < AUDIO_RAG__SECTION__KEY variables
(loader.py:59-93, values converted as in _convert_value 96-116).
"""

import os
from pathlib import Path
from typing import Any

import yaml

from audio_rag_amd.config.schema import AudioRAGConfig
from audio_rag_amd.core.exceptions import ConfigError


def deep_merge(base: dict, override: dict) -> dict:
    result = base.copy()
    for key, value in override.items():
        if key in result and isinstance(result[key], dict) and isinstance(value, dict):
            result[key] = deep_merge(result[key], value)
        else:
            result[key] = value
    return result


def load_yaml(path: Path) -> dict[str, Any]:
    if not path.exists():
        raise ConfigError(f"Config file not found: {path}")
    try:
        with open(path) as f:
            return yaml.safe_load(f) or {}
    except yaml.YAMLError as e:
        raise ConfigError(f"Invalid YAML in {path}: {e}")


def _convert_value(value: str) -> Any:
    low = value.lower()
    if low in ("true", "yes", "1"):
        return True
    if low in ("false", "no", "0"):
        return False
    if low in ("null", "none"):
        return None
    try:
        return float(value) if "." in value else int(value)
    except ValueError:
        return value


def apply_env_overrides(config: dict[str, Any], prefix: str = "AUDIO_RAG") -> dict[str, Any]:
    result = config.copy()
    for key, value in os.environ.items():
        if not key.startswith(f"{prefix}__"):
            continue
        parts = key[len(prefix) + 2:].lower().split("__")
        target = result
        for part in parts[:-1]:
            if part not in target or not isinstance(target[part], dict):
                target[part] = {}
            target = target[part]
        target[parts[-1]] = _convert_value(value)
    return result


def load_config(config_path: Path | str | None = None, env: str | None = None,
                config_dir: Path | str = "configs") -> AudioRAGConfig:
    config_dir = Path(config_dir)
    config: dict[str, Any] = {}
    base_path = config_dir / "base.yaml"
    if base_path.exists():
        config = deep_merge(config, load_yaml(base_path))
    if env:
        env_path = config_dir / f"{env}.yaml"
        if env_path.exists():
            config = deep_merge(config, load_yaml(env_path))
    if config_path:
        config = deep_merge(config, load_yaml(Path(config_path)))
    config = apply_env_overrides(config)
    try:
        return AudioRAGConfig(**config)
    except Exception as e:
        raise ConfigError(f"Configuration validation failed: {e}")
