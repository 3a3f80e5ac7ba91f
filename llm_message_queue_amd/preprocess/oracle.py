"""Exact CPU oracle of the reference preprocessor's text semantics (C10).

Reference: `internal/preprocessor/preprocessor.go`.  What "exact" means here:

* ``strings.Fields`` splits on ``unicode.IsSpace`` -- ASCII ``\\t\\n\\v\\f\\r `` plus
  U+0085, U+00A0 and the Z-category spaces (U+1680, U+2000-200A, U+2028,
  U+2029, U+202F, U+205F, U+3000).  Python's ``str.split()`` also splits on
  U+001C-001F, which Go does not, so it is NOT used.
* ``strings.ToLower`` maps only A-Z, U+212A (KELVIN SIGN -> 'k') and U+0130
  (-> 'i') to ASCII; every other change keeps a character non-ASCII, and all
  the words compared against are ASCII, so that mapping is the one that
  matters.  (Python's ``lower()`` turns U+0130 into "i\\u0307".)
* ``(?i)`` regex literals fold ASCII letters plus the two non-ASCII orbit
  members of ASCII letters: U+017F (long s) ~ 's' and U+212A ~ 'k'.  Counts are
  leftmost non-overlapping occurrences (``FindAllString``).
* ``contains_question``: last byte is '?' (``HasSuffix``, no trimming), or the
  lowered content CONTAINS ``kw + " "`` for kw in what/how/why/when/where/who
  -- substring match, so "somewhat " counts (`preprocessor.go:233-248`).
* Tie in keyword scores: the reference picks by Go map iteration order
  (nondeterministic, defect D17); here the MORE URGENT level wins.
"""
from __future__ import annotations

import re
from typing import Dict, List, Sequence, Tuple

GO_SPACE = frozenset("\t\n\v\f\r \u0085\u00a0\u1680\u2000\u2001\u2002\u2003\u2004"
                     "\u2005\u2006\u2007\u2008\u2009\u200a\u2028\u2029\u202f\u205f\u3000")

POSITIVE_WORDS = ("good", "great", "excellent", "happy", "satisfied")
NEGATIVE_WORDS = ("bad", "terrible", "awful", "angry", "frustrated")
QUESTION_WORDS = ("what", "how", "why", "when", "where", "who")
REALTIME_PATTERNS = ("immediate", "emergency", "asap", "right now")
HIGH_PATTERNS = ("urgent", "important", "priority", "critical", "soon")

# Characters for which our fast GPU path must defer to this oracle: their
# lower-casing or case folding crosses into ASCII.
FOLD_SPECIAL = frozenset("\u017f\u212a\u0130")

_LOWER_MAP = {ord(c): ord(c.lower()) for c in "ABCDEFGHIJKLMNOPQRSTUVWXYZ"}
_LOWER_MAP[0x212A] = ord("k")
_LOWER_MAP[0x0130] = ord("i")
_FOLD_MAP = {ord(c): ord(c.lower()) for c in "ABCDEFGHIJKLMNOPQRSTUVWXYZ"}
_FOLD_MAP[0x017F] = ord("s")
_FOLD_MAP[0x212A] = ord("k")


def sanitize(content: str) -> str:
    """Replace lone surrogates with U+FFFD, as Go's JSON decoder does."""
    try:
        content.encode("utf-8")
        return content
    except UnicodeEncodeError:
        return "".join("\ufffd" if 0xD800 <= ord(c) <= 0xDFFF else c for c in content)


def go_fields(s: str) -> List[str]:
    out, cur = [], []
    for ch in s:
        if ch in GO_SPACE:
            if cur:
                out.append("".join(cur))
                cur = []
        else:
            cur.append(ch)
    if cur:
        out.append("".join(cur))
    return out


def go_lower(s: str) -> str:
    """ToLower restricted to the mappings that can produce ASCII (see module doc)."""
    return s.translate(_LOWER_MAP)


def _fold(s: str) -> str:
    return s.translate(_FOLD_MAP)


class LiteralPattern:
    """A regex that is a plain literal, optionally ``(?i)``-prefixed."""

    __slots__ = ("text", "ci", "source")

    def __init__(self, text: str, ci: bool, source: str):
        self.text = text
        self.ci = ci
        self.source = source

    def count(self, content: str) -> int:
        if not self.text:
            return 0  # empty pattern: not used by the reference
        if self.ci:
            hay, needle = _fold(content), _fold(self.text)
        else:
            hay, needle = content, self.text
        n, i, L = 0, 0, len(needle)
        while True:
            j = hay.find(needle, i)
            if j < 0:
                return n
            n += 1
            i = j + L

    def __repr__(self) -> str:
        return f"LiteralPattern({self.source!r})"


class RegexPattern:
    """Non-literal custom pattern: Python ``re`` stands in for RE2 (documented
    approximation; the default patterns are all literals)."""

    __slots__ = ("rx", "source")

    def __init__(self, source: str):
        src = source
        flags = 0
        if src.startswith("(?i)"):
            flags |= re.IGNORECASE
            src = src[4:]
        self.rx = re.compile(src, flags)
        self.source = source

    def count(self, content: str) -> int:
        return sum(1 for _ in self.rx.finditer(content))

    def __repr__(self) -> str:
        return f"RegexPattern({self.source!r})"


_META = set(".^$*+?()[]{}|\\")


def compile_pattern(pattern: str):
    """Compile like ``regexp.Compile``: literal fast path when possible."""
    ci = pattern.startswith("(?i)")
    body = pattern[4:] if ci else pattern
    if body and not any(c in _META for c in body):
        return LiteralPattern(body, ci, pattern)
    # literal with escaped metacharacters only (e.g. "right\\ now")
    unesc, i, ok = [], 0, True
    while i < len(body):
        c = body[i]
        if c == "\\" and i + 1 < len(body) and body[i + 1] in _META | {" "}:
            unesc.append(body[i + 1])
            i += 2
            continue
        if c in _META:
            ok = False
            break
        unesc.append(c)
        i += 1
    if ok and unesc:
        return LiteralPattern("".join(unesc), ci, pattern)
    return RegexPattern(pattern)


def default_patterns() -> Dict[int, list]:
    return {
        1: [compile_pattern("(?i)" + p) for p in REALTIME_PATTERNS],
        2: [compile_pattern("(?i)" + p) for p in HIGH_PATTERNS],
    }


def keyword_scores(content: str, patterns: Dict[int, Sequence]) -> Dict[int, int]:
    return {prio: sum(p.count(content) for p in pats) for prio, pats in patterns.items()}


def pick_priority(scores: Dict[int, int], default_priority: int) -> int:
    """Highest strictly-positive score; ties -> more urgent (lower int)."""
    best, best_p = 0, default_priority
    for prio in sorted(scores):
        s = scores[prio]
        if s > best:
            best, best_p = s, prio
    return best_p if best > 0 else default_priority


def content_analysis(content: str) -> Tuple[int, str, bool]:
    """(word_count, sentiment, is_question) -- `preprocessor.go:197-249`."""
    words = go_fields(content)
    pos = neg = 0
    for w in words:
        wl = go_lower(w)
        if wl in POSITIVE_WORDS:
            pos += 1
        if wl in NEGATIVE_WORDS:
            neg += 1
    sentiment = "positive" if pos > neg else ("negative" if neg > pos else "neutral")
    return len(words), sentiment, is_question(content)


def is_question(content: str) -> bool:
    if content.endswith("?"):
        return True
    lower = go_lower(content)
    return any((kw + " ") in lower for kw in QUESTION_WORDS)


def sentiment_counts(content: str) -> Tuple[int, int]:
    pos = neg = 0
    for w in go_fields(content):
        wl = go_lower(w)
        pos += wl in POSITIVE_WORDS
        neg += wl in NEGATIVE_WORDS
    return pos, neg


def fnv1a32(data: bytes) -> int:
    h = 0x811C9DC5
    for b in data:
        h ^= b
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


def token_hashes(content: str, max_tokens: int) -> List[int]:
    """FNV-1a-32 of the first <= 32 UTF-8 bytes of each field, ASCII-lowercased
    (the classifier's tokenizer; matches the ``text_analyze`` kernel)."""
    out = []
    for w in go_fields(content):
        b = w.encode("utf-8")[:32]   # the kernel hashes at most 32 bytes per token
        b = bytes((c + 32) if 65 <= c <= 90 else c for c in b)
        out.append(fnv1a32(b))
        if len(out) >= max_tokens:
            break
    return out
