"""TEST INFRASTRUCTURE (rehearsal only): a torch restatement of the plan of
the library's owner-partitioned merge, ``okm_merge_owned``
(orion-kmer_amd/csrc/okm_dist.hip), so that the world-size
2/3 gloo tests run the N>1 orchestration on CPU processes without a GPU.
The product path never imports this file: bench.py and the CLI exchange
through the library's RCCL communicator (okm.Comm).

The plan restated here is the library's:

  1. each rank holds its local table, sorted by key (okm_count's output);
  2. a 2^16-bin histogram of the top key bits is summed over ranks
     (all_reduce) and cut into contiguous, count-balanced key ranges, one per
     rank, by the library's own host split (okm_owner_bounds);
  3. every rank's sorted table splits into contiguous per-owner slices
     (searchsorted on the range boundaries) and all_to_all moves sizes, keys
     and counts (counts as one byte plus escapes, like k_pack_counts);
  4. each owner adds the received sorted runs into one table (weights add:
     the AtomicUsize fetch_add of count.rs:31-34).

The global table is the concatenation of the owners' ranges in rank order.
"""

from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

HIST_BITS = 16

MergeFn = Callable[[torch.Tensor, torch.Tensor], Tuple[torch.Tensor, torch.Tensor]]


class DeviceView:
    """__cuda_array_interface__ of an engine-owned int64 device array, so
    torch.as_tensor(DeviceView(ptr, n), device="cuda") wraps it without a copy."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<i8", "data": (ptr, False),
                                         "version": 3, "strides": None}


def key_bins(keys: torch.Tensor, k: int, bits: int) -> torch.Tensor:
    """Top `bits` bits of the 2k-bit keys (int64 view of u64 keys)."""
    shift = 2 * k - bits
    b = keys >> shift if shift > 0 else keys
    return b & ((1 << bits) - 1)


def hist_bits(k: int) -> int:
    return min(HIST_BITS, 2 * k)


def local_histogram(keys: torch.Tensor, k: int) -> torch.Tensor:
    """Instances per top-`bits` bin of a SORTED table: one searchsorted of the
    2^bits bin starts (a few microseconds) instead of a bincount over every
    key (the engine's tables are sorted, count.rs:119)."""
    bits = hist_bits(k)
    nb = 1 << bits
    if keys.numel() == 0:
        return torch.zeros(nb, dtype=torch.int64, device=keys.device)
    starts = torch.arange(nb, dtype=torch.int64, device=keys.device) << (2 * k - bits)
    cuts = torch.searchsorted(_order_view(keys, k), _order_view(starts, k), right=False)
    ends = torch.cat([cuts[1:], torch.tensor([keys.numel()], dtype=torch.int64, device=keys.device)])
    return ends - cuts


def owner_ranges(hist: np.ndarray, world: int) -> List[int]:
    """Bin boundaries b_0=0 <= b_1 <= ... <= b_world=len(hist): rank r owns
    bins [b_r, b_{r+1}); cuts where the running total first reaches r/world.
    The library's host split (okm_owner_bounds, the same code okm_merge_owned
    runs), so the gloo tests exercise it."""
    from okm import owner_bounds
    return owner_bounds(np.asarray(hist, dtype=np.uint64), world)


def _order_view(keys: torch.Tensor, k: int) -> torch.Tensor:
    """int64 values whose signed order equals the keys' unsigned order."""
    if k < 32:
        return keys
    return keys ^ torch.tensor(-(1 << 63), dtype=torch.int64, device=keys.device)


def exchange(keys: torch.Tensor, counts: torch.Tensor, k: int,
             group: Optional[dist.ProcessGroup] = None) -> Tuple[torch.Tensor, torch.Tensor, List[int]]:
    """Move every (key, count) of this rank's sorted table to the owner of its
    key range; returns the received concatenated runs and the bin bounds."""
    rk, rc, bounds, _ = exchange_runs(keys, counts, k, group)
    return rk, rc, bounds


def shared_bounds(tables: Sequence[torch.Tensor], k: int,
                  group: Optional[dist.ProcessGroup] = None) -> List[int]:
    """Owner bin bounds balanced over the sum of several sorted tables (one
    all_reduce): tables exchanged with the same bounds land on the same owner
    key by key, so per-owner results combine by a plain sum (C5's |A ∩ B|)."""
    world = dist.get_world_size(group)
    hist = local_histogram(tables[0], k)
    for t in tables[1:]:
        hist += local_histogram(t, k)
    dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
    return owner_ranges(hist.cpu().numpy(), world)


def exchange_runs(keys: torch.Tensor, counts: Optional[torch.Tensor], k: int,
                  group: Optional[dist.ProcessGroup] = None, bounds: Optional[List[int]] = None,
                  narrow_counts: bool = True):
    """exchange(), also returning the number of pairs received from each rank:
    rank r's run is rk[sum(sizes[:r]) : sum(sizes[:r+1])], sorted by key
    (okm_add_sorted_pairs_device takes each run without copying).  counts may
    be None (sets: rc is then None); bounds default to this table's own
    balanced ranges (shared_bounds() for several tables); narrow_counts sends
    counts as bytes with escapes (_send_counts_u8), the received rc is int64
    either way."""
    world = dist.get_world_size(group)
    dev = keys.device
    if bounds is None:
        bounds = shared_bounds([keys], k, group)
    bits = hist_bits(k)
    shift = 2 * k - bits
    # key boundaries of the owners' ranges (first key of each range); a bound
    # equal to the bin count is +infinity (b << shift would wrap to 0 at k=32)
    nbins = 1 << bits
    kb = []
    for b in bounds[1:-1]:
        v = min(b, nbins - 1) << shift
        if v >= 1 << 63:
            v -= 1 << 64
        kb.append(v)
    kb_t = torch.tensor(kb, dtype=torch.int64, device=dev)
    if world > 1:
        cuts = torch.searchsorted(_order_view(keys, k), _order_view(kb_t, k), right=False)
        past = torch.tensor([b >= nbins for b in bounds[1:-1]], dtype=torch.bool, device=dev)
        cuts = torch.where(past, torch.full_like(cuts, keys.numel()), cuts)
    else:
        cuts = torch.zeros(0, dtype=torch.int64, device=dev)
    edges = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), cuts,
                       torch.tensor([keys.numel()], dtype=torch.int64, device=dev)])
    send_sizes = (edges[1:] - edges[:-1]).to(torch.int64)
    recv_sizes = torch.empty_like(send_sizes)
    dist.all_to_all_single(recv_sizes, send_sizes, group=group)
    ss = send_sizes.cpu().tolist()
    rs = recv_sizes.cpu().tolist()
    rk = torch.empty(sum(rs), dtype=torch.int64, device=dev)
    dist.all_to_all_single(rk, keys.contiguous(), rs, ss, group=group)
    rc = None
    if counts is not None:
        if narrow_counts:
            rc = _send_counts_u8(counts.contiguous(), edges, ss, rs, group)
        else:
            rc = torch.empty(sum(rs), dtype=torch.int64, device=dev)
            dist.all_to_all_single(rc, counts.contiguous(), rs, ss, group=group)
    return rk, rc, bounds, rs


COUNT_ESCAPE = 255


def _send_counts_u8(counts: torch.Tensor, edges: torch.Tensor, ss: List[int], rs: List[int],
                    group: Optional[dist.ProcessGroup]) -> torch.Tensor:
    """Counts over the wire as one byte each: the count's low byte (one cast
    pass, no clamp), and a count >= 256 also travels as an escape entry (its
    position in the destination's run and its full value) that overwrites
    the byte on arrival.  Tables of covered reads hold mostly small counts, so a pair costs
    9 bytes instead of 16 on the link; xGMI is point-to-point (one link per GPU
    pair), so at 2 and 4 ranks these bytes bound the exchange."""
    world = len(ss)
    dev = counts.device
    r8 = torch.empty(sum(rs), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(r8, counts.to(torch.uint8), rs, ss, group=group)  # low byte (wraps)
    esc = torch.nonzero(counts > COUNT_ESCAPE).flatten()  # ascending positions
    esend = (torch.searchsorted(esc, edges[1:]) - torch.searchsorted(esc, edges[:-1])).to(torch.int64)
    erecv = torch.empty_like(esend)
    dist.all_to_all_single(erecv, esend, group=group)
    es, er = esend.cpu().tolist(), erecv.cpu().tolist()
    ranks = torch.arange(world, dtype=torch.int64, device=dev)
    rel = esc - edges[:-1][torch.repeat_interleave(ranks, esend)]  # position within its destination run
    rrel = torch.empty(sum(er), dtype=torch.int64, device=dev)
    rval = torch.empty(sum(er), dtype=torch.int64, device=dev)
    dist.all_to_all_single(rrel, rel, er, es, group=group)
    dist.all_to_all_single(rval, counts[esc], er, es, group=group)
    rc = r8.to(torch.int64)
    if sum(er):
        run0 = torch.tensor(np.concatenate([[0], np.cumsum(rs[:-1], dtype=np.int64)]), dtype=torch.int64,
                            device=dev)
        rc[run0[torch.repeat_interleave(ranks, erecv)] + rrel] = rval
    return rc


UnionFn = Callable[[torch.Tensor, List[int]], Tuple[int, object]]
IntersectFn = Callable[[object, int, object, int], int]


def distributed_compare(a_keys: torch.Tensor, b_keys: torch.Tensor, k: int, union: UnionFn,
                        intersect: IntersectFn,
                        group: Optional[dist.ProcessGroup] = None) -> Tuple[int, int, int]:
    """compare.rs:51-66 over ranks (SURVEY.md §8(e) "C5"): a_keys / b_keys are
    this rank's union of its share of DB1's / DB2's references (sorted unique
    keys).  Both go to value-range owners under ONE set of bounds, each owner
    unions its received runs (union(received, run sizes) -> (size, handle))
    and intersects its two owned ranges; the three sizes are summed with one
    all_reduce.  Returns (|A|, |B|, |A ∩ B|) of the global unions."""
    bounds = shared_bounds([a_keys, b_keys], k, group)
    ra, _, _, rsa = exchange_runs(a_keys, None, k, group, bounds)
    na, ha = union(ra, rsa)
    rb, _, _, rsb = exchange_runs(b_keys, None, k, group, bounds)
    nb, hb = union(rb, rsb)
    inter = intersect(ha, na, hb, nb)
    dev = a_keys.device
    tot = torch.tensor([na, nb, inter], dtype=torch.int64, device=dev)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=group)
    na_g, nb_g, i_g = (int(x) for x in tot.cpu().tolist())
    return na_g, nb_g, i_g


def distributed_merge(keys: torch.Tensor, counts: torch.Tensor, k: int, merge: MergeFn,
                      group: Optional[dist.ProcessGroup] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Steps 2-4 above; returns this rank's owned range of the global table."""
    rk, rc, _ = exchange(keys, counts, k, group)
    return merge(rk, rc)


def gather_global(keys: torch.Tensor, counts: torch.Tensor,
                  group: Optional[dist.ProcessGroup] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Concatenate every owner's range in rank order on every rank (tests and
    small outputs only; a CLI writes each range in order instead)."""
    world = dist.get_world_size(group)
    n = torch.tensor([keys.numel()], dtype=torch.int64, device=keys.device)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    mx = int(max(int(x.item()) for x in ns))
    pk = torch.zeros(mx, dtype=torch.int64, device=keys.device)
    pc = torch.zeros(mx, dtype=torch.int64, device=keys.device)
    pk[:keys.numel()] = keys
    pc[:counts.numel()] = counts
    gk = [torch.empty_like(pk) for _ in range(world)]
    gc = [torch.empty_like(pc) for _ in range(world)]
    dist.all_gather(gk, pk, group=group)
    dist.all_gather(gc, pc, group=group)
    ok = np.concatenate([g[:int(c.item())].cpu().numpy() for g, c in zip(gk, ns)]).view(np.uint64)
    oc = np.concatenate([g[:int(c.item())].cpu().numpy() for g, c in zip(gc, ns)]).view(np.uint64)
    return ok, oc
