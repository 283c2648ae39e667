"""One process per GPU without an external launcher.

``python3 bench.py --gpus N`` (no ``WORLD_SIZE`` in the environment) must
measure N GPUs, the same as ``torch.distributed.run --nproc-per-node N
bench.py --gpus N`` does (BASELINE ``metric``: bases/s "at 1/2/4/8 MI355X";
SURVEY.md §8(e)), or fail loudly.  This module is that launcher:

* :func:`probe_devices` counts the visible HIP devices in a CHILD process, so
  the launching process makes no HIP call before it starts the ranks (a
  process that has initialised the GPU must not fork/exec the ranks);
* :func:`spawn_ranks` starts N children with the ``torch.distributed`` env
  (``RANK``, ``LOCAL_RANK``, ``WORLD_SIZE``, ``LOCAL_WORLD_SIZE``,
  ``MASTER_ADDR=127.0.0.1``, ``MASTER_PORT``), each in its own process group,
  relays rank 0's stdout (the driver's one JSON line) to this process's
  stdout, sends the other ranks' stdout to stderr, and returns non-zero as
  soon as any rank fails (the survivors, which would otherwise block in
  their next collective, are terminated by process group).

Nothing here imports torch or loads the engine library.
"""

from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import List, Optional, Sequence

_AMD = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    """A free TCP port on 127.0.0.1 for the rendezvous."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def probe_devices(timeout: float = 120.0) -> int:
    """Visible HIP devices, counted by a child process (hipGetDeviceCount
    through the engine library); 0 when the library or the runtime is
    missing."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import okm\n"
            "print(okm.device_count())\n") % _AMD
    try:
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout)
    except (OSError, subprocess.TimeoutExpired):
        return 0
    if r.returncode != 0:
        return 0
    try:
        return max(0, int(r.stdout.strip().splitlines()[-1]))
    except (ValueError, IndexError):
        return 0


def rank_env(rank: int, world: int, port: int, base: Optional[dict] = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # RCCL / device-tensor sharing across processes: the hosts here only do dmabuf IPC
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _killpg(p: subprocess.Popen, sig: int) -> None:
    try:
        os.killpg(p.pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def _stop_all(procs: Sequence[subprocess.Popen], grace_s: float) -> None:
    live = [p for p in procs if p.poll() is None]
    for p in live:
        _killpg(p, signal.SIGTERM)
    t_end = time.time() + grace_s
    for p in live:
        try:
            p.wait(timeout=max(0.0, t_end - time.time()))
        except subprocess.TimeoutExpired:
            _killpg(p, signal.SIGKILL)
            p.wait()


def spawn_ranks(cmd: Sequence[str], world: int, grace_s: float = 10.0, poll_s: float = 0.05,
                stdout=None) -> int:
    """Run `cmd` as `world` ranks (one process each) and wait for all of
    them.  Returns 0 when every rank exits 0; otherwise the first failing
    rank's exit status (a signal-killed rank gives 128 + signal), after
    SIGTERM (then, past `grace_s`, SIGKILL) to the process groups of the
    ranks still running."""
    if world < 1:
        raise ValueError("world must be >= 1")
    out = stdout if stdout is not None else sys.stdout
    port = free_port()
    procs: List[subprocess.Popen] = []
    relay: Optional[threading.Thread] = None
    try:
        for r in range(world):
            p = subprocess.Popen(list(cmd), env=rank_env(r, world, port),
                                 stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(),
                                 start_new_session=True)
            procs.append(p)
            if r == 0:
                def pump(src=p.stdout):
                    for line in iter(src.readline, b""):
                        out.write(line.decode(errors="replace"))
                        out.flush()
                relay = threading.Thread(target=pump, daemon=True)
                relay.start()
    except OSError:
        for p in procs:
            _killpg(p, signal.SIGKILL)
        raise
    rc = 0
    failed = None
    try:
        while True:
            alive = 0
            for r, p in enumerate(procs):
                s = p.poll()
                if s is None:
                    alive += 1
                elif s != 0 and failed is None:
                    failed = r
                    rc = s if s > 0 else 128 - s
            if failed is not None or alive == 0:
                break
            time.sleep(poll_s)
        if failed is not None:
            sys.stderr.write(f"launch: rank {failed} exited with status {rc}; stopping the other ranks\n")
    finally:
        # a failing rank, Ctrl-C or any error in this process: every rank still
        # running is stopped by process group (each rank has its own session, so
        # the terminal's signal never reaches it), SIGTERM then SIGKILL
        _stop_all(procs, grace_s)
    if relay is not None:
        relay.join(timeout=grace_s)
    return rc


def launch_or_none(gpus: int, cmd: Sequence[str], what: str = "bench.py") -> Optional[int]:
    """The launcher decision: None when this process is already one rank of
    a job (``WORLD_SIZE`` set by torch.distributed.run or by spawn_ranks) or
    a single-GPU run; otherwise the exit status of running `cmd` as `gpus`
    ranks, or 2 with a message when fewer devices are visible than ranks
    asked for (one rank per GPU: RCCL refuses two ranks on one device)."""
    if "WORLD_SIZE" in os.environ or gpus <= 1:
        return None
    n_dev = probe_devices()
    if gpus > n_dev:
        sys.stderr.write(f"{what}: --gpus {gpus} asks for {gpus} ranks, {n_dev} device"
                         f"{'' if n_dev == 1 else 's'} visible (one rank per GPU)\n")
        return 2
    return spawn_ranks(cmd, gpus)
