"""CPU codec of the k<=64 extension (restatement-defined; no reference):
MSB-first 2-bit encoding over 2k bits, reverse complement, canonical min —
checked against plain Python integer arithmetic and the C oracle."""

import random

import okm
from oracle import load as oracle_load

import ctypes


def py_encode(seq: bytes) -> int:
    v = 0
    for b in seq:
        v = (v << 2) | "ACGT".index(chr(b).upper())
    return v


def py_rc(v: int, k: int) -> int:
    r = 0
    for _ in range(k):
        r = (r << 2) | ((v & 3) ^ 3)
        v >>= 2
    return r


def test_u128_codec_matches_python_and_oracle():
    rnd = random.Random(7)
    lib = oracle_load()
    for _ in range(300):
        k = rnd.randint(1, 64)
        seq = bytes(rnd.choice(b"ACGTacgt") for _ in range(k))
        v = okm.seq_to_u128(seq, k)
        assert v == py_encode(seq)
        out = (ctypes.c_uint64 * 2)()
        assert lib.oracle_seq_to_u128(seq, k, k, out) == 1 and (out[1] << 64 | out[0]) == v
        assert okm.u128_to_seq(v, k) == seq.upper()
        assert okm.reverse_complement_u128(v, k) == py_rc(v, k)
        assert okm.canonical_u128(v, k) == min(v, py_rc(v, k))
        if k <= 32:  # agrees with the reference-pinned u64 codec
            assert v == okm.seq_to_u64(seq, k)
            assert okm.canonical_u128(v, k) == okm.canonical_u64(v, k)
    assert okm.seq_to_u128(b"ACGN" + b"A" * 40, 44) is None
    assert okm.seq_to_u128(b"A" * 65, 65) is None
    # all-T k=64 canonicalises to all-A: ~0 is never a key (the empty sentinel)
    assert okm.canonical_u128((1 << 128) - 1, 64) == 0
