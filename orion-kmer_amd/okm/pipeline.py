"""The N>1 count step: every rank counts its own batch, then the per-rank
tables merge by key-range owner (the reference's single map
over all input, count.rs:48,52-89, drained and sorted once, :106-119).

Reads shard by record, so each rank counts its shard with no communication;
the one exchange is the library's ``okm_merge_owned`` (csrc/okm_dist.hip:
HIP histogram / pack / unpack kernels, grouped ncclSend/ncclRecv over xGMI,
the owner's count of the received sorted slices).  This module is the host
orchestration around it that ``bench.py`` runs at N>1:

* :func:`run_pipelined` overlaps the counts of the next batches (worker
  threads, one local context each plus one spare, taken in turn) with the
  exchange + merge of batch i (this thread, the only one that issues
  collectives, so every rank issues them in one order);
* :class:`OwnedCountPipeline` is that loop over ``okm.Comm`` and
  ``okm.KmerCounter`` objects, with the failure agreement the merge needs:
  a rank whose count failed still joins the step's one-word all-reduce, and
  when any rank reports a failure EVERY rank raises before the merge
  (``okm_merge_owned`` would otherwise re-run the failed count, or merge
  partial input, on the failing rank only, and its peers would block in the
  next step's collectives).

The communicator may be RCCL (``Comm(world, rank, uid, device)``, one process
per GPU) or the loopback transport (``Comm.init_loopback(P)``: P ranks on
threads of one process, one device) — the tests drive the same class both
ways, and the CPU tests drive it over gloo with a restated exchange.
Nothing here imports torch.
"""

from __future__ import annotations

import queue
import threading
from typing import Callable, List, Optional, Sequence


class PeerFailure(RuntimeError):
    """Raised on a rank whose own step succeeded when a peer's count failed."""


def run_pipelined(nsteps: int, count_into: Callable[[int, int], object],
                  consume: Callable[[int, int, object, Callable[[], None]], object],
                  finish: Optional[Callable[[int, int, object], object]] = None,
                  workers: int = 1, nbuf: int = 2) -> List[object]:
    """Pipelined step loop.  `workers` threads count batches (count_into(i, j)
    -> handle, batch i into table buffer j = i % nbuf; steps are taken in
    order, and a buffer is reused only after consume released it) while this
    thread consumes them in step order (consume(i, j, handle, release) ->
    result), so the exchange of batch i overlaps the counts of the next
    batches.  consume calls release() once the table may be reused.  Only this
    thread issues collectives, so every rank issues them in the same order.
    workers <= nbuf - 1 keeps one buffer for the batch being consumed.

    With `finish`, consume's result is a payload handed to a third thread that
    runs finish(i, m, payload) -> result on merge slot m = i % 2 (no
    collectives there): the finish of batch i then overlaps the exchange of
    batch i + 1 and the count of batch i + 2, and the slot is reused by batch
    i + 2 only after its finish returned.  Results are in step order either
    way.  An exception in any thread is re-raised here."""
    workers = max(1, min(workers, max(1, nbuf - 1)))
    free = [threading.Semaphore(1) for _ in range(nbuf)]
    done: dict = {}
    cv = threading.Condition()
    nxt = [0]
    err: List[BaseException] = []
    stop = threading.Event()

    def acquire(sem: "threading.Semaphore") -> bool:
        while not sem.acquire(timeout=0.1):
            if stop.is_set():
                return False
        return True

    def producer():
        try:
            while not stop.is_set():
                with cv:
                    i = nxt[0]
                    if i >= nsteps:
                        return
                    nxt[0] += 1
                if not acquire(free[i % nbuf]):
                    return
                h = count_into(i, i % nbuf)
                with cv:
                    done[i] = h
                    cv.notify_all()
        except BaseException as e:  # surfaced on the consuming thread
            with cv:
                err.append(e)
                stop.set()
                cv.notify_all()

    out: List[object] = [None] * nsteps
    mfree = [threading.Semaphore(1), threading.Semaphore(1)]
    mq: "queue.Queue" = queue.Queue()

    def finisher():
        try:
            while True:
                item = mq.get()
                if item is None:
                    return
                i, m, payload = item
                out[i] = finish(i, m, payload)
                mfree[m].release()
        except BaseException as e:
            err.append(e)
            stop.set()

    ths = [threading.Thread(target=producer, daemon=True) for _ in range(workers)]
    for th in ths:
        th.start()
    fth = threading.Thread(target=finisher, daemon=True) if finish is not None else None
    if fth is not None:
        fth.start()
    try:
        for i in range(nsteps):
            with cv:
                while i not in done and not err:
                    cv.wait(timeout=0.1)
                if err:
                    break
                h = done.pop(i)
            j = i % nbuf
            r = consume(i, j, h, free[j].release)
            if fth is None:
                out[i] = r
                continue
            if not acquire(mfree[i % 2]):
                break
            mq.put((i, i % 2, r))
    finally:
        if fth is not None:
            mq.put(None)
            fth.join()
        stop.set()
        for th in ths:
            th.join()
    if err:
        raise err[0]
    return out


def agree_or_raise(comm, failure: Optional[BaseException], what: str = "count") -> None:
    """Collective: every rank learns whether any rank's `what` failed (one
    all-reduced word) and, if so, every rank raises — the failing rank its
    own exception, the others PeerFailure — so no rank is left alone in a
    later collective."""
    bad = comm.allreduce([1 if failure is not None else 0])[0]
    if failure is not None:
        raise failure
    if bad:
        raise PeerFailure(f"{bad} peer rank(s) failed their {what}; every rank stops at this step")


def comm_audit(infos: Sequence[dict], world: int) -> dict:
    """The N>1 line's proof of what ran: every rank's ``Comm.info()``
    (gathered by the caller, rank order) summarised -- the communicator size
    the library holds (okm_comm_size), the ranks the transport itself
    reports (RCCL's ncclCommCount / ncclCommUserRank / ncclCommCuDevice) and
    each rank's device PCI bus id.  ``ok``: `world` ranks, every one agreeing
    on it, the transport reporting `world` ranks with ranks 0..world-1, and
    (RCCL) `world` distinct PCI devices -- N ranks were N GPUs."""
    infos = list(infos)
    sizes = sorted({int(i["size"]) for i in infos})
    tranks = sorted({int(i["transport_ranks"]) for i in infos})
    transports = sorted({str(i["transport"]) for i in infos})
    pci = [str(i["pci_bus_id"]) for i in infos]
    distinct = len(set(p for p in pci if p))
    ok = (len(infos) == world and sizes == [world] and tranks == [world]
          and sorted(int(i["transport_rank"]) for i in infos) == list(range(world))
          and sorted(int(i["rank"]) for i in infos) == list(range(world)))
    if transports == ["rccl"]:
        ok = ok and distinct == world
    return {"comm_ranks": sizes[0] if len(sizes) == 1 else sizes,
            "transport": transports[0] if len(transports) == 1 else transports,
            "transport_ranks": tranks[0] if len(tranks) == 1 else tranks,
            "distinct_pci_bus_ids": distinct,
            "ranks": [{"rank": int(i["rank"]), "device": int(i["device"]), "pci_bus_id": str(i["pci_bus_id"]),
                       "transport_rank": int(i["transport_rank"]),
                       "transport_device": int(i["transport_device"])} for i in infos],
            "ok": bool(ok)}


class OwnedCountPipeline:
    """bench.py's N>1 step loop: per step, reset + add this
    rank's batch (``add_batch(counter, step)``) + ``okm_count`` into one of
    workers + 1 local contexts (`workers` counting threads, each context its
    own HIP stream), then ``okm_merge_owned`` of that table into one of two
    owner contexts.  The counts of the next steps overlap the exchange + merge
    of step i (:func:`run_pipelined`).  Each step returns this rank's owned
    distinct count; after :meth:`run` the owner context of the last step
    (:meth:`owned`) holds this rank's key range of the global table, and the
    ranks' ranges in rank order ARE the sorted table of every rank's batch.

    `counter` makes a context (``lambda: okm.KmerCounter(k, "count",
    device)``); `comm` is an ``okm.Comm`` (RCCL or loopback) or anything with
    ``allreduce`` and ``merge_owned``."""

    def __init__(self, comm, counter: Callable[[], object], add_batch: Callable[[object, int], None],
                 workers: int = 1):
        self.comm = comm
        self.add_batch = add_batch
        self.workers = max(1, workers)
        self.local = [counter() for _ in range(self.workers + 1)]  # one more than the counting threads
        self.owners = [counter(), counter()]
        self.phase_ms = {"exchange": 0.0, "merge": 0.0}  # okm_comm_last_times, summed over steps
        self._last = 0

    def count_one(self, c, i: int) -> int:
        c.reset()
        self.add_batch(c, i)
        return c.count()

    def warm(self) -> None:
        """Count one batch into every local context (device pools sized before
        a timed region; no collectives)."""
        for c in self.local:
            self.count_one(c, 0)

    def run(self, nsteps: int, first_step: int = 0) -> List[int]:
        def count_into(i, j):
            try:
                return self.count_one(self.local[j], first_step + i)
            except Exception as e:  # handed to the merge thread's agreement
                return e

        def consume(i, j, counted, release):
            try:
                agree_or_raise(self.comm, counted if isinstance(counted, BaseException) else None)
                n = self.comm.merge_owned(self.local[j], self.owners[i % 2])
            finally:
                release()
            self._last = i % 2
            last_times = getattr(self.comm, "last_times", None)
            if last_times is not None:
                t = last_times()
                self.phase_ms["exchange"] += t["plan_ms"] + t["exchange_ms"]
                self.phase_ms["merge"] += t["merge_ms"]
            return n

        return run_pipelined(nsteps, count_into, consume, workers=self.workers, nbuf=len(self.local))

    def owned(self):
        """The owner context of the last merged step."""
        return self.owners[self._last]

    def contexts(self) -> Sequence[object]:
        return list(self.local) + list(self.owners)

    def close(self) -> None:
        for c in self.contexts():
            close = getattr(c, "close", None)
            if close is not None:
                close()
