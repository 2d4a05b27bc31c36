"""File helpers behind the data API.

* ``csv_to_json`` — apps/data/util/csv_handler.py:5-21 (DictReader rows -> list of dicts)
* ``dir_tree`` — apps/data/util/file_walker.py:5-31 (file -> its name, dir -> nested dict)
* ``safe_join`` — path-traversal guard the reference lacked (``relative_path`` was
  concatenated into a filesystem path unchecked, apps/data/views.py:242; quirk 8)
* ``timestamped_name`` — apps/data/views.py:66-86 (``<stem>_<YYYYmmddHHMMSS>.<ext>``)
"""
from __future__ import annotations

import csv
import json
import os
import time
from typing import Any, Dict, List, Optional


def csv_to_rows(path: str) -> List[Dict[str, str]]:
    with open(path, newline="", encoding="utf-8", errors="replace") as f:
        reader = csv.DictReader(f)
        return [dict(r) for r in reader]


def csv_to_json(path: str) -> str:
    return json.dumps(csv_to_rows(path), ensure_ascii=False)


def dir_tree(path: str) -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for name in sorted(os.listdir(path)):
        p = os.path.join(path, name)
        out[name] = dir_tree(p) if os.path.isdir(p) else name
    return out


def safe_join(root: str, rel: Optional[str]) -> Optional[str]:
    """Join ``rel`` under ``root``; None if it would escape ``root``."""
    root_abs = os.path.realpath(root)
    if not rel:
        return root_abs
    p = os.path.realpath(os.path.join(root_abs, rel))
    if p != root_abs and not p.startswith(root_abs + os.sep):
        return None
    return p


def timestamped_name(name: str, now: Optional[float] = None) -> str:
    ts = time.strftime("%Y%m%d%H%M%S", time.localtime(time.time() if now is None else now))
    parts = name.split(".")
    if len(parts) == 1:
        return f"{parts[0]}_{ts}"
    return ".".join(parts[:-1]) + f"_{ts}." + parts[-1]


def valid_name(name: Optional[str]) -> bool:
    """Model / file names: the reference routes only matched ``\\w+`` (urls.py); we also
    reject path separators and dot-names everywhere a name becomes a directory."""
    if not name or len(name) > 128 or name in (".", ".."):
        return False
    return all(c.isalnum() or c in "_-." for c in name) and not name.startswith(".")
