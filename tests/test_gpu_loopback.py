"""The product multi-GPU merge (okm_merge_owned, okm_dist.hip) at P > 1 ranks
on ONE device, through the loopback transport (okm_comm_init_loopback): the
same owner plan, k_pack_counts / k_widen_counts / k_apply_escapes kernels,
message pieces and owner merge as over RCCL, with the exchange done by device
copies between P virtual ranks driven from P host threads.

The reference's semantics are one map over all the input (count.rs:48),
drained, filtered and sorted once (count.rs:106-119): the owners' ranges in
rank order must equal the oracle's table of the whole input, exactly.  Sets
(build.rs:46-58) and the distributed compare (compare.rs:51-66) likewise."""

import os
import threading

import numpy as np
import pytest

import okm
from okm import testing
from oracle import OracleCounter

pytestmark = pytest.mark.gpu
# a rank that never reaches a collective ends it after a minute, not five


@pytest.fixture(autouse=True)
def _loopback_timeout():
    """A rank that never arrives ends a collective after 60 s, not 300 (the
    conftest resets every knob after each test)."""
    testing.set_knob("loopback_timeout_ms", 60_000)
    yield


def run_ranks(P, fn):
    """fn(rank) on P threads (one per virtual rank); returns the results in
    rank order, re-raising the first exception."""
    out, err = [None] * P, [None] * P

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException as e:  # surfaced below
            err[r] = e

    th = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
        assert not t.is_alive(), "a virtual rank hung"
    for e in err:
        if e is not None:
            raise e
    return out


def _records(n, genome, seed, hot_every=0, read_len=150):
    b = okm.synth_reads(n, read_len, genome_len=genome, genome_seed=seed, seed=seed)
    recs = b.reshape(n, read_len + 1)
    if hot_every:
        recs[::hot_every, :read_len] = ord("A")  # a hot key: counts far past the one-byte escape
    return recs


def _shards(recs, P, empty_rank=None):
    """Contiguous record shards (count.rs:23-38 is per record); empty_rank gets none."""
    ranks = [r for r in range(P) if r != empty_rank]
    parts = np.array_split(recs, len(ranks))
    out = [np.zeros(0, np.uint8)] * P
    for r, p in zip(ranks, parts):
        out[r] = np.ascontiguousarray(p).reshape(-1)
    return out


def _oracle(recs, k):
    oc = OracleCounter(k)
    oc.add_separated(np.ascontiguousarray(recs).reshape(-1))
    return oc.result(1)


def _merge_case(P, k, shards, owner_mode, mode="count", wide=False):
    """Every rank counts its shard and merges; returns [(keys, counts, n_owned)]."""
    comms = okm.Comm.init_loopback(P, 0)

    def rank(r):
        local = okm.KmerCounter(k, mode, wide=wide)
        owner = local if owner_mode == "local" else okm.KmerCounter(k, mode, wide=wide)
        buf = None
        try:
            if len(shards[r]):
                buf = okm.DeviceBuffer(len(shards[r]))
                buf.upload(shards[r])
                local.add_device_batch(buf.address, len(shards[r]))
            n = comms[r].merge_owned(local, owner)
            keys, counts = owner.result(1)
            return keys, counts, n, comms[r].last_bytes()
        finally:
            if buf is not None:
                buf.free()
            local.close()
            if owner is not local:
                owner.close()

    try:
        return run_ranks(P, rank)
    finally:
        for c in comms:
            c.close()


def _check_ranges(res, ek, ec, with_counts=True):
    keys = np.concatenate([r[0] for r in res])
    assert np.array_equal(keys, ek)  # the owners' ranges in rank order ARE the sorted global table
    if with_counts:
        counts = np.concatenate([r[1] for r in res])
        assert np.array_equal(counts, ec)
    assert [r[2] for r in res] == [len(r[0]) for r in res]
    for a, b in zip(res, res[1:]):  # contiguous, ascending, disjoint ranges
        if len(a[0]) and len(b[0]):
            assert a[0][-1] < b[0][0]


@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("owner_mode", ["separate", "local"])
def test_loopback_merge_exact(P, owner_mode):
    k = 31
    recs = _records(60_000, 300_000, 21, hot_every=40)
    ek, ec = _oracle(recs, k)
    assert ec.max() > 255
    res = _merge_case(P, k, _shards(recs, P), owner_mode)
    _check_ranges(res, ek, ec)
    # traffic: every rank moves (P-1)/P of its table, 9 B per pair + escapes
    sent = sum(r[3][0] for r in res)
    recv = sum(r[3][1] for r in res)
    assert sent == recv > 0


@pytest.mark.parametrize("P", [3, 8])
def test_loopback_merge_empty_rank(P):
    k = 27
    recs = _records(20_000, 200_000, 22, hot_every=25)
    ek, ec = _oracle(recs, k)
    res = _merge_case(P, k, _shards(recs, P, empty_rank=1), "separate")
    _check_ranges(res, ek, ec)


def test_loopback_merge_k32_top_bin():
    """k = 32: canonical keys with the top 16 bits all ones (TTTTTTTT...AAAAAAAA
    windows) land in the last histogram bin; ~0 is never a key."""
    k, P = 32, 3
    rng = np.random.default_rng(5)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    top = [b"TTTTTTTT" + acgt[rng.integers(0, 4, 16)].tobytes() + b"AAAAAAAA" for _ in range(3000)]
    rnd = [acgt[rng.integers(0, 4, 60)].tobytes() for _ in range(3000)]
    recs = top + rnd + [b"T" * 40, b"A" * 40] * 50
    rng.shuffle(recs)
    oc = OracleCounter(k)
    oc.add_records(recs)
    ek, ec = oc.result(1)
    assert (ek >> np.uint64(48) == 0xFFFF).sum() >= 1000
    data = [b"\n".join(recs[r::P]) + b"\n" for r in range(P)]
    shards = [np.frombuffer(d, np.uint8).copy() for d in data]
    res = _merge_case(P, k, shards, "separate")
    # the records were dealt round-robin: same multiset
    _check_ranges(res, ek, ec)
    assert (res[-1][0] >> np.uint64(48) == 0xFFFF).any()


@pytest.mark.parametrize("P", [3, 8])
def test_loopback_merge_set_mode(P):
    k = 21
    recs = _records(30_000, 400_000, 23)
    ek, _ = _oracle(recs, k)
    res = _merge_case(P, k, _shards(recs, P), "separate", mode="set")
    _check_ranges(res, ek, None, with_counts=False)


@pytest.mark.parametrize("piece", [4096, 65536])
def test_loopback_merge_multi_piece(monkeypatch, piece):
    """Tiny message pieces (knob piece_bytes): every message (keys, count bytes, escapes) splits
    into many pieces, grouped by piece index on every rank."""
    testing.set_knob("piece_bytes", piece)
    k, P = 31, 3
    recs = _records(40_000, 250_000, 24, hot_every=30)
    ek, ec = _oracle(recs, k)
    res = _merge_case(P, k, _shards(recs, P), "separate")
    _check_ranges(res, ek, ec)
    assert max(r[3][0] for r in res) > 20 * piece  # really many pieces


def test_loopback_owner_takes_more_input_after_merge():
    """After okm_merge_owned the owner holds no pointer into the local table or
    the communicator: local is reset and refilled, the comm merges
    again, and then the owner counts more input on top of its range."""
    k, P = 25, 2
    recs = _records(30_000, 300_000, 25, hot_every=50)
    extra = _records(5_000, 300_000, 26)
    comms = okm.Comm.init_loopback(P, 0)
    shards = _shards(recs, P)

    def rank(r):
        with okm.KmerCounter(k) as local, okm.KmerCounter(k) as owner, okm.KmerCounter(k) as other:
            buf = okm.DeviceBuffer(len(shards[r]))
            buf.upload(shards[r])
            local.add_device_batch(buf.address, len(shards[r]))
            comms[r].merge_owned(local, owner)
            mine_k, mine_c = owner.result(1)
            # overwrite everything the owner could still point at
            local.reset()
            local.add_device_batch(buf.address, len(shards[r]))
            comms[r].merge_owned(local, other)
            buf.free()
            e = np.ascontiguousarray(extra).reshape(-1)
            owner.add_records([bytes(x) for x in e.tobytes().split(b"\n") if x], normalized=True)
            gk, gc = owner.result(1)
            return mine_k, mine_c, gk, gc

    try:
        res = run_ranks(P, rank)
    finally:
        for c in comms:
            c.close()
    ek, ec = _oracle(recs, k)
    assert np.array_equal(np.concatenate([r[0] for r in res]), ek)
    xk, xc = _oracle(extra, k)
    for mk, mc, gk, gc in res:
        want = {}
        for a, b in zip(mk.tolist(), mc.tolist()):
            want[a] = want.get(a, 0) + b
        for a, b in zip(xk.tolist(), xc.tolist()):
            want[a] = want.get(a, 0) + b
        wk = np.array(sorted(want), dtype=np.uint64)
        wc = np.array([want[x] for x in wk.tolist()], dtype=np.uint64)
        assert np.array_equal(gk, wk) and np.array_equal(gc, wc)


def test_loopback_failure_agreement(monkeypatch):
    """A rank failing between collectives (knob fail_rank: out of memory
    while sizing its receive buffers) makes EVERY rank return an error, and the
    communicator still merges afterwards."""
    k, P = 21, 3
    recs = _records(10_000, 100_000, 27)
    shards = _shards(recs, P)
    comms = okm.Comm.init_loopback(P, 0)
    testing.set_knob("fail_rank", 1)

    def attempt(r):
        with okm.KmerCounter(k) as local, okm.KmerCounter(k) as owner:
            buf = okm.DeviceBuffer(len(shards[r]))
            buf.upload(shards[r])
            local.add_device_batch(buf.address, len(shards[r]))
            buf.free()
            try:
                comms[r].merge_owned(local, owner)
                return None
            except okm.OkmError as e:
                return e.status

    try:
        st = run_ranks(P, attempt)
        assert st[1] == okm._lib.OKM_E_NOMEM
        assert st[0] == st[2] == okm._lib.OKM_E_COMM
        testing.set_knob("fail_rank", -1)
        assert run_ranks(P, attempt) == [None] * P
    finally:
        for c in comms:
            c.close()


def test_loopback_missing_rank_times_out(monkeypatch):
    """A rank that never joins the collective ends it with OKM_E_COMM on the
    others (no hang), and the aborted communicator refuses later merges."""
    testing.set_knob("loopback_timeout_ms", 2000)
    comms = okm.Comm.init_loopback(2, 0)
    try:
        with okm.KmerCounter(15) as local, okm.KmerCounter(15) as owner:
            local.add_records([b"ACGTACGTTGCAGGATCCAT" * 5])
            with pytest.raises(okm.OkmError) as ei:
                comms[0].merge_owned(local, owner)
            assert ei.value.status == okm._lib.OKM_E_COMM
            with pytest.raises(okm.OkmError):
                comms[0].merge_owned(local, owner)
    finally:
        for c in comms:
            c.close()


@pytest.mark.parametrize("P", [2, 8])
def test_loopback_distributed_compare(P):
    """compare.rs:51-66 over P ranks through okm_merge_owned_n (set mode, one
    owner split for both DBs): each rank unions its share of every DB's
    references, both unions go to the same key-range owners, each owner
    intersects its two ranges on the device, and |A|, |B|, |A∩B| are summed."""
    k = 31
    samples = [_records(6_000, 200_000 + 50_000 * (s % 3), 900 + (s % 5)).reshape(-1) for s in range(12)]
    half = len(samples) // 2
    comms = okm.Comm.init_loopback(P, 0)

    def rank(r):
        a = okm.KmerCounter(k, "set")
        b = okm.KmerCounter(k, "set")
        oa = okm.KmerCounter(k, "set")
        ob = okm.KmerCounter(k, "set")
        try:
            for s in range(r, len(samples), P):  # samples dealt round-robin
                dst = a if s < half else b
                buf = okm.DeviceBuffer(len(samples[s]))
                buf.upload(samples[s])
                dst.add_device_batch(buf.address, len(samples[s]))
                buf.free()
            return okm.distributed_compare(comms[r], a, b, oa, ob)
        finally:
            for c in (a, b, oa, ob):
                c.close()

    try:
        res = run_ranks(P, rank)
    finally:
        for c in comms:
            c.close()
    sets = [_oracle(s.reshape(-1, 151), k)[0] for s in samples]
    A = np.unique(np.concatenate(sets[:half]))
    B = np.unique(np.concatenate(sets[half:]))
    inter = len(np.intersect1d(A, B, assume_unique=True))
    for got in res:  # every rank holds the summed sizes
        assert got == (len(A), len(B), inter)
    assert 0 < inter < min(len(A), len(B))


@pytest.mark.parametrize("P", [2, 8])
@pytest.mark.parametrize("sparse", [False, True])
def test_loopback_wire_formats(monkeypatch, P, sparse):
    """Keys on the wire as u64 and as 5-byte deltas (knob wire_deltas forced),
    with key escapes for gaps >= 2^40: most gaps of a ~100 K-key table
    escape; counts past the byte escape.  Both formats give the oracle's
    table."""
    k = 31
    recs = _records(1_500 if sparse else 40_000, 2_000_000 if sparse else 300_000, 28 + P,
                    hot_every=0 if sparse else 35)
    ek, ec = _oracle(recs, k)
    for deltas in ("1", "0"):
        testing.set_knob("wire_deltas", int(deltas))
        res = _merge_case(P, k, _shards(recs, P), "separate")
        _check_ranges(res, ek, ec)


@pytest.mark.parametrize("P", [2, 4])
def test_loopback_wire_deltas_dense_table_bytes(monkeypatch, P):
    """A table of ~14 M keys (gaps ~2^37 of the 2^61 canonical 31-mers): the
    default wire format at 2-4 ranks is the 5-byte deltas, and both formats
    give the same owner ranges.  Measured 7.1 B per pair against 9: keys with
    first base T are ~1/7 as dense as those with A (canonical skew), so there
    ~1/3 of the gaps pass 2^40 and escape; a C3 shard table (~1.4 G keys,
    gaps ~2^31) hardly escapes at all (6 B per pair)."""
    k = 31
    recs = _records(1_000_000, 10_000_000, 30)
    sent, tables = {}, {}
    for deltas in ("", "0"):
        testing.set_knob("wire_deltas", int(deltas) if deltas else -1)
        res = _merge_case(P, k, _shards(recs, P), "separate")
        sent[deltas] = sum(r[3][0] for r in res)
        tables[deltas] = (np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res]))
    assert np.array_equal(tables[""][0], tables["0"][0]) and np.array_equal(tables[""][1], tables["0"][1])
    assert len(tables["0"][0]) > 10_000_000
    assert bool((tables["0"][0][1:] > tables["0"][0][:-1]).all())
    assert sent[""] < 0.82 * sent["0"], sent


def test_loopback_wire_deltas_multi_piece_set_mode(monkeypatch):
    """5-byte keys cut into odd-sized pieces (a key straddles two pieces), set mode."""
    testing.set_knob("wire_deltas", 1)
    testing.set_knob("piece_bytes", 4104)
    k, P = 27, 3
    recs = _records(25_000, 500_000, 29)
    ek, _ = _oracle(recs, k)
    res = _merge_case(P, k, _shards(recs, P), "local", mode="set")
    _check_ranges(res, ek, None, with_counts=False)


# ---------------------------------------------------------------------------
# k > 32 (K128 keys, the two-u64 extension of BASELINE configs[3]): the keys
# cross as u64 word pairs (never 5-byte deltas); the same plan, count bytes,
# escapes and owner merge
# ---------------------------------------------------------------------------

def _oracle_wide(recs, k):
    from oracle import OracleCounterWide
    oc = OracleCounterWide(k)
    oc.add_separated_range(np.ascontiguousarray(recs).reshape(-1), 0, 0, 1)  # 0 key bits: every key
    return oc.result(1)


def _check_ranges_wide(res, ek, ec):
    keys = np.concatenate([r[0].reshape(-1, 2) for r in res])
    assert np.array_equal(keys, ek)  # rank order = the sorted global table
    assert np.array_equal(np.concatenate([r[1] for r in res]), ec)
    assert [r[2] for r in res] == [len(r[1]) for r in res]
    ints = [okm.keys128_to_int(r[0]) for r in res]
    for a, b in zip(ints, ints[1:]):  # contiguous, ascending, disjoint ranges
        if a and b:
            assert a[-1] < b[0]


@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("k,owner_mode", [(45, "separate"), (63, "local"), (63, "separate")])
def test_loopback_merge_wide_exact(P, k, owner_mode):
    recs = _records(20_000, 200_000, 31, hot_every=30)
    ek, ec = _oracle_wide(recs, k)
    assert ec.max() > 255  # counts past the one-byte escape
    res = _merge_case(P, k, _shards(recs, P), owner_mode, wide=True)
    _check_ranges_wide(res, ek, ec)
    sent = sum(r[3][0] for r in res)
    assert sent == sum(r[3][1] for r in res) > 0


def test_loopback_merge_wide_multi_piece_empty_rank(monkeypatch):
    """Small pieces split every 16-B-key message (a piece boundary may fall
    between a key's two words: the pieces count u64 words), plus an empty rank;
    wire_deltas = 1 must not apply to K128 keys."""
    testing.set_knob("piece_bytes", 4104)
    testing.set_knob("wire_deltas", 1)
    k, P = 63, 3
    recs = _records(15_000, 150_000, 32, hot_every=20)
    ek, ec = _oracle_wide(recs, k)
    res = _merge_case(P, k, _shards(recs, P, empty_rank=2), "separate", wide=True)
    _check_ranges_wide(res, ek, ec)
    assert max(r[3][0] for r in res) > 20 * 4104
