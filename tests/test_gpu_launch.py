"""More ranks / GPUs than devices fails loudly on a real box (VERDICT r4
item 1): `python3 bench.py --gpus N` without WORLD_SIZE launches one rank per
GPU itself, and with fewer devices than N it must exit non-zero at once
instead of reporting one GPU's number as N's; the CLI's `count --gpus N`
likewise (okm_group_create: one context per GPU)."""

import os
import subprocess
import sys
import time

import pytest

import okm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "orion-kmer_amd", "build", "orion-kmer")

pytestmark = pytest.mark.gpu


def test_bench_more_ranks_than_devices_fails_fast():
    n = okm.device_count()
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n + 1), "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert f"{n + 1} ranks, {n} device" in r.stderr
    assert r.stdout == ""
    assert time.time() - t0 < 60


def test_cli_count_more_gpus_than_devices_fails(tmp_path):
    n = okm.device_count()
    fa = tmp_path / "a.fa"
    fa.write_bytes(b">r\nACGTACGTAC\n")
    out = tmp_path / "o.tsv"
    r = subprocess.run([CLI, "count", "-k", "3", "-i", str(fa), "-o", str(out), "--gpus", str(n + 1)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 1, (r.returncode, r.stderr)
    assert f"{n + 1} GPUs asked, {n} visible" in r.stderr
    # the device range is checked too: --device D --gpus 1 with D past the last device
    r = subprocess.run([CLI, "count", "-k", "3", "-i", str(fa), "-o", str(out), "--device", str(n), "--gpus", "1"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 1, (r.returncode, r.stderr)
