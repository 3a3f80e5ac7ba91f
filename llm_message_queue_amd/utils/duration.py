"""Go ``time.Duration`` text parsing/formatting (viper decodes "100ms", "5m", "1h30m").

Reference: the duration-typed config fields, e.g. ``max_wait_time``,
``monitor_interval``, ``process_interval`` (`pkg/config/config.go:49-68`), so
`configs/config.yaml` loads unchanged."""
from __future__ import annotations

import re
from typing import Any

_UNITS_NS = {
    "ns": 1, "us": 1_000, "µs": 1_000, "μs": 1_000, "ms": 1_000_000,
    "s": 1_000_000_000, "m": 60_000_000_000, "h": 3_600_000_000_000,
}
_TOKEN = re.compile(r"([0-9]*\.?[0-9]+)(ns|us|µs|μs|ms|s|m|h)")


def parse_duration_ns(value: Any) -> int:
    """Parse a Go duration string (or a bare number of ns) into integer ns."""
    if value is None:
        return 0
    if isinstance(value, bool):
        raise ValueError(f"invalid duration {value!r}")
    if isinstance(value, (int, float)):
        return int(value)
    s = str(value).strip()
    if s in ("", "0"):
        return 0
    sign = 1
    if s[0] in "+-":
        sign = -1 if s[0] == "-" else 1
        s = s[1:]
    pos, total = 0, 0.0
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise ValueError(f"invalid duration {value!r}")
        total += float(m.group(1)) * _UNITS_NS[m.group(2)]
        pos = m.end()
    return sign * int(round(total))


def parse_duration_s(value: Any) -> float:
    return parse_duration_ns(value) / 1e9


def format_duration_ns(ns: int) -> str:
    """Compact Go-style rendering (``1m30s``, ``100ms``)."""
    ns = int(ns)
    if ns == 0:
        return "0s"
    neg = ns < 0
    ns = abs(ns)
    if ns < 1_000:
        out = f"{ns}ns"
    elif ns < 1_000_000:
        out = f"{ns / 1e3:g}µs"
    elif ns < 1_000_000_000:
        out = f"{ns / 1e6:g}ms"
    else:
        h, rem = divmod(ns, 3_600_000_000_000)
        m, rem = divmod(rem, 60_000_000_000)
        sec = rem / 1e9
        out = (f"{h}h" if h else "") + (f"{m}m" if (m or h) else "") + f"{sec:g}s"
    return ("-" if neg else "") + out
