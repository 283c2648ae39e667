"""Test hooks of the engine (include/orion_kmer_testing.h): process-wide
knobs that force the rare paths (overflowed sampled capacities, key-range
groups, tiny message pieces, a failing rank ...) so the tests can check them
against the oracle at small sizes.  Not for production use."""

from __future__ import annotations

import contextlib
from typing import Dict, Iterator

from . import _lib

KNOBS: Dict[str, int] = {
    "l1_cap_permille": 0,
    "part_cap_permille": 1,
    "part_max_bits": 2,
    "group_keys": 3,
    "group_exact": 4,
    "sorted_path": 5,
    "wire_deltas": 6,
    "piece_bytes": 7,
    "fail_rank": 8,
    "loopback_timeout_ms": 9,
    "tsv_chunk": 10,
    "gz_par_min_bytes": 11,
    "gz_chunk_bytes": 12,
    "gz_strict": 13,
    "no_libdeflate": 14,
    "hbm_budget_bytes": 15,
    "group_over": 16,
}


def set_knob(name: str, value: int) -> None:
    """value < 0 (or None) unsets the knob."""
    _lib.load().okm_test_set(KNOBS[name], -1 if value is None else int(value))


def get_knob(name: str) -> int:
    return int(_lib.load().okm_test_get(KNOBS[name]))


def reset_all() -> None:
    for name in KNOBS:
        set_knob(name, -1)


@contextlib.contextmanager
def knobs(**values: int) -> Iterator[None]:
    """Set knobs for the duration of a with-block (restoring their values)."""
    old = {n: get_knob(n) for n in values}
    try:
        for n, v in values.items():
            set_knob(n, v)
        yield
    finally:
        for n, v in old.items():
            set_knob(n, v)
