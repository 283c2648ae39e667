"""bench.py's own multi-rank launcher (okm/launch.py) on the CPU.

`python3 bench.py --gpus N` without WORLD_SIZE must run N rank processes
(one per GPU) or fail loudly, never report one GPU as N (BASELINE metric "at
1/2/4/8 MI355X").  These tests drive the launcher with a
stub rank (tests/launch_stub.py) that stops before any GPU call, and
bench.py itself on this GPU-less container, where asking for 2 ranks must
fail within seconds.
"""

import io
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orion-kmer_amd"))

from okm import launch  # noqa: E402

STUB = os.path.join(ROOT, "tests", "launch_stub.py")


def _env(monkeypatch, tmp_path, **kv):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("STUB_DIR", str(tmp_path))
    for k, v in kv.items():
        monkeypatch.setenv(k, v)


def test_children_get_rank_env_and_rank0_line_is_relayed(monkeypatch, tmp_path):
    _env(monkeypatch, tmp_path)
    out = io.StringIO()
    rc = launch.spawn_ranks([sys.executable, STUB, "--gpus", "3"], 3, stdout=out)
    assert rc == 0
    lines = [l for l in out.getvalue().splitlines() if l.strip()]
    assert len(lines) == 1, lines  # only rank 0's stdout is relayed
    line = json.loads(lines[0])
    assert line["argv"] == ["--gpus", "3"]
    e0 = line["env"]
    assert e0["RANK"] == "0" and e0["LOCAL_RANK"] == "0" and e0["WORLD_SIZE"] == "3"
    assert e0["LOCAL_WORLD_SIZE"] == "3" and e0["MASTER_ADDR"] == "127.0.0.1"
    assert e0["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    for r in (1, 2):
        with open(tmp_path / f"rank{r}.json") as fh:
            er = json.load(fh)
        assert er["RANK"] == str(r) and er["LOCAL_RANK"] == str(r) and er["WORLD_SIZE"] == "3"
        assert er["MASTER_PORT"] == e0["MASTER_PORT"]  # one rendezvous


def test_failing_rank_fails_the_run_and_stops_the_others(monkeypatch, tmp_path):
    _env(monkeypatch, tmp_path, STUB_FAIL_RANK="1", STUB_FAIL_AFTER="0.5", STUB_HANG="1")
    t0 = time.time()
    rc = launch.spawn_ranks([sys.executable, STUB], 3, grace_s=5.0, stdout=io.StringIO())
    assert rc == 3
    # the hanging ranks were terminated, not waited for (they sleep 600 s)
    assert time.time() - t0 < 60


def test_interrupted_launcher_stops_every_rank(monkeypatch, tmp_path):
    """Ctrl-C (or any error) in the launching process must not leave the
    ranks running: each has its own session, so the terminal's SIGINT never
    reaches them, and ranks blocked in a collective would hold their GPUs."""
    _env(monkeypatch, tmp_path, STUB_HANG="1")
    real_sleep = time.sleep

    def interrupt_once_started(s):
        if all((tmp_path / f"rank{r}.json").exists() for r in (1, 2)):
            raise KeyboardInterrupt
        real_sleep(s)

    monkeypatch.setattr(launch.time, "sleep", interrupt_once_started)
    t0 = time.time()
    try:
        launch.spawn_ranks([sys.executable, STUB], 3, grace_s=5.0, stdout=io.StringIO())
        raise AssertionError("the interrupt must propagate")
    except KeyboardInterrupt:
        pass
    monkeypatch.setattr(launch.time, "sleep", real_sleep)
    assert time.time() - t0 < 60
    for r in (1, 2):
        with open(tmp_path / f"rank{r}.json") as fh:
            pid = json.load(fh)["pid"]
        deadline = time.time() + 10
        while time.time() < deadline:
            try:
                os.kill(pid, 0)  # still there (or a zombie not yet reaped by init)?
            except ProcessLookupError:
                break
            with open(f"/proc/{pid}/stat") as st:
                if st.read().split()[2] == "Z":
                    break
            real_sleep(0.1)
        else:
            raise AssertionError(f"rank {r} (pid {pid}) still running after the launcher was interrupted")


def test_failing_rank0_fails_the_run(monkeypatch, tmp_path):
    _env(monkeypatch, tmp_path, STUB_FAIL_RANK="0")
    assert launch.spawn_ranks([sys.executable, STUB], 2, grace_s=5.0, stdout=io.StringIO()) == 3


def test_launch_is_a_noop_inside_a_rank_or_at_one_gpu(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert launch.launch_or_none(4, ["false"]) is None
    monkeypatch.delenv("WORLD_SIZE")
    assert launch.launch_or_none(1, ["false"]) is None


def test_more_ranks_than_devices_is_an_error(monkeypatch, capsys):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(launch, "probe_devices", lambda timeout=120.0: 1)
    assert launch.launch_or_none(2, ["false"]) == 2
    assert "2 ranks, 1 device visible" in capsys.readouterr().err


def test_bench_gpus_2_without_devices_fails_fast():
    """This container has no GPU: bench.py --gpus 2 must exit non-zero with
    the rank/device message within seconds, having started no rank."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "2 ranks, 0 devices visible" in r.stderr
    assert r.stdout == ""
    assert time.time() - t0 < 60


def test_bench_world_size_disagreeing_with_gpus_is_an_error():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "--gpus 2 but WORLD_SIZE=1" in r.stderr
