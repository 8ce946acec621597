"""Token-stream text deltas that never split a UTF-8 character.

Mirrors core/src/streaming.rs:1-80 (``extract_delta``, ``DeltaTracker``): the CLI and the
server decode the whole generated prefix after every token and emit only the new suffix; a
trailing U+FFFD (an incomplete multi-byte character) is held back until a later token or the
final flush completes it.
"""
from __future__ import annotations

REPLACEMENT = "�"


def extract_delta(previous: str, current: str) -> str:
    """streaming.rs:4-18: suffix of ``current`` after its common prefix with ``previous``."""
    if current.startswith(previous):
        return current[len(previous):]
    n = 0
    for a, b in zip(previous, current):
        if a != b:
            break
        n += 1
    return current[n:]


class DeltaTracker:
    """streaming.rs:21-70."""

    def __init__(self):
        self.previous = ""

    def reset(self):
        self.previous = ""

    def advance(self, current: str, is_final: bool) -> str:
        delta = extract_delta(self.previous, current)
        if not delta:
            self.previous = current
            return delta
        if not is_final:
            idx = delta.find(REPLACEMENT)
            if idx == 0:
                return ""
            if idx > 0:
                delta = delta[:idx]
                self.previous += delta
                return delta
        self.previous = current
        return delta

    def snapshot(self) -> str:
        return self.previous


def decode_ids(tokenizer, ids) -> str:
    """``tokenizer.decode(ids, skip_special_tokens=true)`` over the ids that fit u32
    (the reference's ``filter_map(u32::try_from)``, cli/src/app.rs:174-178)."""
    toks = [int(t) for t in ids if 0 <= int(t) < 2 ** 32]
    if not toks:
        return ""
    try:
        return tokenizer.decode(toks, skip_special_tokens=True)
    except TypeError:
        return tokenizer.decode(toks)
