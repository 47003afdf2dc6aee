"""GUI preference persistence (same file and API as the reference's session.py:15-41)."""
from __future__ import annotations

import json
from pathlib import Path
from typing import Any, Optional

_SESSION_FILE = Path.home() / ".nightcore_analyzer_session.json"


def _load() -> dict:
    try:
        return json.loads(_SESSION_FILE.read_text(encoding="utf-8"))
    except Exception:
        return {}


def _save(data: dict) -> None:
    try:
        _SESSION_FILE.write_text(json.dumps(data, indent=2), encoding="utf-8")
    except Exception:
        pass


def get(key: str, default: Any = None) -> Any:
    return _load().get(key, default)


def set(key: str, value: Any) -> None:  # noqa: A001 - reference API name
    data = _load()
    data[key] = value
    _save(data)


def set_many(updates: Optional[dict] = None, **kwargs: Any) -> None:
    """Persist every pair of ``updates`` in one write (session.py:37-41); keyword pairs are
    accepted too."""
    data = _load()
    data.update(updates or {})
    data.update(kwargs)
    _save(data)
