"""The multi-GPU merge inside the library (okm_dist.hip): okm_comm over RCCL
and okm_merge_owned, through the C ABI.  The GPU box has one MI355X, so the
communicator here has one rank (RCCL self send/recv: every pack, send/recv,
unpack and merge step runs, the owner range is the whole key space); the N>1
split is covered by the CPU tests of okm_owner_bounds (test_host_abi.py) and
the gloo tests (test_dist_gloo.py), and measured by the driver's 8-GPU run.
Exact against the local table and the oracle (count.rs:48, one map)."""

import ctypes

import numpy as np
import pytest

import okm
import restate as R
from okm import testing
from oracle import OracleCounter

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm1():
    c = okm.Comm(1, 0, okm.comm_unique_id(), 0)
    assert c.rank == 0 and c.size == 1
    yield c
    c.close()


def test_comm_info_rccl_reports_itself(comm1):
    """okm_comm_get_info over real RCCL: what bench.py's N>1 `comm` object is
    built from -- RCCL's own rank count / rank / device and the PCI bus id."""
    from okm.pipeline import comm_audit
    i = comm1.info()
    assert i["transport"] == "rccl" and i["size"] == 1 and i["rank"] == 0 and i["device"] == 0
    assert i["transport_ranks"] == 1 and i["transport_rank"] == 0 and i["transport_device"] == 0
    assert len(i["pci_bus_id"]) >= 7 and ":" in i["pci_bus_id"]
    a = comm_audit([i], 1)
    assert a["ok"] and a["distinct_pci_bus_ids"] == 1
    assert not comm_audit([i, dict(i, rank=1, transport_rank=1)], 2)["ok"]  # 2 ranks on one GPU: refused


def _batch(n, genome, seed):
    return okm.synth_reads(n, 150, genome_len=genome, genome_seed=seed, seed=seed)


@pytest.mark.parametrize("genome", [10_000, 2_000_000])   # 10 kb: counts far past the 255 byte escape
def test_merge_owned_single_rank_equals_local(comm1, genome):
    k = 31
    b = _batch(200_000, genome, 7)
    ref = OracleCounter(k)
    ref.add_separated(b)
    ek, ec = ref.result(1)
    assert (ec > 255).any() == (genome == 10_000)
    buf = okm.DeviceBuffer(len(b))
    buf.upload(b)
    with okm.KmerCounter(k) as local, okm.KmerCounter(k) as owner:
        local.add_device_batch(buf.address, len(b))
        lk, lc = local.result(1)  # the local table before the merge
        n = comm1.merge_owned(local, owner)
        gk, gc = owner.result(1)
        t = comm1.last_times()
        # one rank: the local's table was handed to the owner (okm_engine.hip
        # adopt_result: no copy) and the local left reset
        assert local.count() == 0
        # again, after a new count: the owner is reset, the local's pool swapped back
        local.add_device_batch(buf.address, len(b))
        assert comm1.merge_owned(local, owner) == n
        g2k, g2c = owner.result(1)
        # the owner keeps its table as input: one more add merges into it (count.rs:48)
        owner.add_device_batch(buf.address, len(b))
        o3k, o3c = owner.result(1)
    buf.free()
    assert n == len(ek)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert np.array_equal(lk, ek) and np.array_equal(lc, ec)
    assert np.array_equal(g2k, ek) and np.array_equal(g2c, ec)
    assert np.array_equal(o3k, ek) and np.array_equal(o3c, 2 * ec)
    assert t["plan_ms"] >= 0 and t["exchange_ms"] >= 0 and t["merge_ms"] >= 0


@pytest.mark.parametrize("piece", [4096])  # (1 MiB pieces dropped in round 6: 4 KiB covers more pieces)
def test_merge_owned_rccl_multi_piece(comm1, monkeypatch, piece):
    """Real RCCL at one rank with every message cut into many pieces
    (test knob piece_bytes): keys, count bytes and escapes of the self slice."""
    testing.set_knob("piece_bytes", piece)
    k = 31
    b = _batch(200_000, 3_000_000, 8)
    b.reshape(200_000, 151)[::50, :150] = ord("A")  # a hot key: counts past the one-byte escape
    ref = OracleCounter(k)
    ref.add_separated(b)
    ek, ec = ref.result(1)
    assert (ec > 255).any() and len(ek) * 8 > 16 * piece
    buf = okm.DeviceBuffer(len(b))
    buf.upload(b)
    with okm.KmerCounter(k) as ctx:
        ctx.add_device_batch(buf.address, len(b))
        assert comm1.merge_owned(ctx, ctx) == len(ek)
        gk, gc = ctx.result(1)
    buf.free()
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


def test_merge_owned_set_mode(comm1):
    k = 21
    b = _batch(50_000, 300_000, 3)
    ref = OracleCounter(k)
    ref.add_separated(b)
    ek, _ = ref.result(1)
    with okm.KmerCounter(k, "set") as local, okm.KmerCounter(k, "set") as owner:
        local.add_records([bytes(r) for r in b.tobytes().split(b"\n") if r], normalized=True)
        assert comm1.merge_owned(local, owner) == len(ek)
        gk, _ = owner.result(1)
    assert np.array_equal(gk, ek)


def test_merge_owned_k32_and_empty(comm1):
    # k = 32 (unsigned key order, the top histogram bin) and an empty local table
    with okm.KmerCounter(32) as local, okm.KmerCounter(32) as owner:
        local.add_records([b"T" * 40, b"A" * 40, b"ACGT" * 20])
        ref = OracleCounter(32)
        ref.add_records([b"T" * 40, b"A" * 40, b"ACGT" * 20])
        ek, ec = ref.result(1)
        assert comm1.merge_owned(local, owner) == len(ek)
        gk, gc = owner.result(1)
        assert np.array_equal(gk, ek) and np.array_equal(gc, ec)
    with okm.KmerCounter(25) as local, okm.KmerCounter(25) as owner:
        assert comm1.merge_owned(local, owner) == 0


def test_comm_init_all_one_device():
    (c,) = okm.Comm.init_all([0])
    with okm.KmerCounter(15) as local, okm.KmerCounter(15) as owner:
        local.add_records([b"ACGTTGCAACGTAGCTAGCTAGGATCGA" * 10])
        nl = local.count()
        n = c.merge_owned(local, owner)
        assert n == nl == owner.count()  # (one rank: the local's table moved to the owner)
    c.close()


def test_merge_owned_argument_errors(comm1):
    with okm.KmerCounter(21) as a, okm.KmerCounter(25) as b:
        with pytest.raises(okm.OkmError):
            comm1.merge_owned(a, b)  # k mismatch
    with okm.KmerCounter(45, wide=True) as a, okm.KmerCounter(63, wide=True) as b:
        with pytest.raises(okm.OkmError):
            comm1.merge_owned(a, b)  # k mismatch among K128 contexts


@pytest.mark.parametrize("piece", ["", "4104"])  # 4,104 B = 513 words: pieces split keys' word pairs
def test_merge_owned_wide_rccl(comm1, monkeypatch, piece):
    """k = 63 (K128 keys): the slices cross RCCL as u64 word pairs, the owner
    counts them; exact against the restatement (one rank: self send/recv)."""
    if piece:
        testing.set_knob("piece_bytes", int(piece))
    from oracle import OracleCounterWide
    k = 63
    b = _batch(30_000, 200_000, 9)
    b.reshape(30_000, 151)[::20, :150] = ord("A")  # a hot key: counts past the one-byte escape
    ref = OracleCounterWide(k)
    ref.add_separated_range(b, 0, 0, 1)
    ek, ec = ref.result(1)
    assert (ec > 255).any()
    buf = okm.DeviceBuffer(len(b))
    buf.upload(b)
    # owner == local: the table goes through an RCCL self send/recv (K128 word
    # pairs, cut into pieces by the knob) -- a separate owner would take it
    # as it stands at one rank (adopt_result)
    with okm.KmerCounter(k, wide=True) as ctx:
        ctx.add_device_batch(buf.address, len(b))
        n = comm1.merge_owned(ctx, ctx)
        gk, gc = ctx.result(1)
        sent, recv = comm1.last_bytes()
    buf.free()
    assert n == len(ec)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)
    assert sent == recv == 0  # one rank: only the self slice, nothing crosses a link


def test_merge_owned_into_local_context(comm1):
    # owner == local: the counting context takes its own range back
    k = 27
    b = _batch(100_000, 500_000, 4)
    ref = OracleCounter(k)
    ref.add_separated(b)
    ek, ec = ref.result(1)
    with okm.KmerCounter(k) as ctx:
        ctx.add_records([bytes(r) for r in b.tobytes().split(b"\n") if r], normalized=True)
        assert comm1.merge_owned(ctx, ctx) == len(ek)
        gk, gc = ctx.result(1)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)


def _group_count(k, batches, n_gpus, min_count=1):
    lib = okm._lib.load()
    g = ctypes.c_void_p()
    okm._lib.check(lib.okm_group_create(ctypes.byref(g), k, 0, n_gpus, None, 0), "okm_group_create")
    try:
        for b in batches:
            data, offs = okm.pack_records([bytes(r) for r in b.tobytes().split(b"\n") if r])
            okm._lib.check(lib.okm_group_add_batch(g, data.ctypes.data, offs.ctypes.data, len(offs) - 1, 1),
                           "okm_group_add_batch")
        nd = ctypes.c_uint64()
        okm._lib.check(lib.okm_group_count(g, ctypes.byref(nd)), "okm_group_count")
        kp, cp, n = ctypes.POINTER(ctypes.c_uint64)(), ctypes.POINTER(ctypes.c_uint64)(), ctypes.c_uint64()
        okm._lib.check(lib.okm_group_finish_counts(g, min_count, ctypes.byref(kp), ctypes.byref(cp), ctypes.byref(n)),
                       "okm_group_finish_counts")
        keys = np.ctypeslib.as_array(kp, shape=(n.value,)).copy() if n.value else np.zeros(0, np.uint64)
        counts = np.ctypeslib.as_array(cp, shape=(n.value,)).copy() if n.value else np.zeros(0, np.uint64)
        lib.okm_free_result(kp)
        lib.okm_free_result(cp)
        assert lib.okm_group_size(g) >= 1 and lib.okm_group_owner(g, 0)
        return nd.value, keys, counts
    finally:
        lib.okm_group_destroy(g)


@pytest.mark.parametrize("n_gpus", [1, 0])  # 0: every visible device (one on the box)
def test_group_pipelined_count(n_gpus):
    k = 31
    batches = [_batch(40_000, 400_000, 10 + i) for i in range(5)]
    ref = OracleCounter(k)
    for b in batches:
        ref.add_separated(b)
    ek, ec = ref.result(1)
    nd, gk, gc = _group_count(k, batches, n_gpus)
    assert nd == len(ek)
    assert np.array_equal(gk, ek) and np.array_equal(gc, ec)
    _, fk, fc = _group_count(k, batches, n_gpus, min_count=3)
    sel = ec >= 3
    assert np.array_equal(fk, ek[sel]) and np.array_equal(fc, ec[sel])


@pytest.mark.parametrize("ext,chunk", [("tsv", "1500"), ("tsv", ""), ("tsv.gz", "4096"), ("tsv.zst", "")])
def test_group_write_counts_tsv_streamed(tmp_path, monkeypatch, ext, chunk):
    """okm_group_write_counts_tsv: the table streamed off the GPU in chunks
    (test knob tsv_chunk: entries) equals count.rs:127-135's TSV of the oracle table,
    filtered by min_count, also when it overwrites a LONGER existing file
    (written in place, then cut to length)."""
    if chunk:
        testing.set_knob("tsv_chunk", int(chunk))
    k = 21
    batches = [_batch(20_000, 300_000, 50 + i) for i in range(3)]
    ref = OracleCounter(k)
    for b in batches:
        ref.add_separated(b)
    lib = okm._lib.load()
    for m in (1, 2):
        ek, ec = ref.result(m)
        want = "".join(f"{okm.u64_to_seq(int(x), k).decode()}\t{int(c)}\n" for x, c in zip(ek, ec)).encode()
        out = tmp_path / f"o{m}.{ext}"
        if ext == "tsv":
            out.write_bytes(b"X" * (len(want) + 12345))  # stale longer content
        g = ctypes.c_void_p()
        okm._lib.check(lib.okm_group_create(ctypes.byref(g), k, 0, 1, None, 0), "okm_group_create")
        try:
            for b in batches:
                data, offs = okm.pack_records([bytes(r) for r in b.tobytes().split(b"\n") if r])
                okm._lib.check(lib.okm_group_add_batch(g, data.ctypes.data, offs.ctypes.data, len(offs) - 1, 1),
                               "okm_group_add_batch")
            nl = ctypes.c_uint64()
            okm._lib.check(lib.okm_group_write_counts_tsv(g, str(out).encode(), m, ctypes.byref(nl)),
                           "okm_group_write_counts_tsv")
        finally:
            lib.okm_group_destroy(g)
        assert nl.value == len(ek)
        raw = R.decompress_by_extension(str(out), out.read_bytes())
        assert raw == want, m
