"""Minimal stand-in for python-fire's flag parsing (fire is not installed):
`--name value`, `--name=value`, dashes == underscores, positional args kept in
order; values parsed like fire (bool / int / float / str)."""
from __future__ import annotations

from typing import Any, Dict, List, Tuple


def _value(s: str) -> Any:
    if s in ("True", "true"):
        return True
    if s in ("False", "false"):
        return False
    if s in ("None", "none"):
        return None
    for cast in (int, float):
        try:
            return cast(s)
        except ValueError:
            pass
    return s


def parse(argv: List[str]) -> Tuple[List[Any], Dict[str, Any]]:
    pos, kw = [], {}
    i = 0
    while i < len(argv):
        a = argv[i]
        if a.startswith("--"):
            key = a[2:]
            if "=" in key:
                key, val = key.split("=", 1)
                kw[key.replace("-", "_")] = _value(val)
            elif i + 1 < len(argv) and not argv[i + 1].startswith("--"):
                kw[key.replace("-", "_")] = _value(argv[i + 1])
                i += 1
            else:
                kw[key.replace("-", "_")] = True
        else:
            pos.append(_value(a))
        i += 1
    return pos, kw
