"""The orion-kmer CLI's host-side contract (cli.rs / main.rs): flags, usage
errors (exit 2), the reference's error strings (exit 1), no GPU needed."""

import os
import subprocess

import numpy as np

import pytest

from conftest import has_gpu
from okm import _lib


def run(*args):
    return subprocess.run([_lib.CLI_PATH, *args], capture_output=True, text=True, timeout=60)


def test_version_and_help():
    r = run("--version")
    assert r.returncode == 0 and r.stdout.strip() == "orion-kmer 0.1.0"
    r = run("count", "--help")
    assert r.returncode == 0 and "--kmer-size" in r.stdout and "--input-files" in r.stdout
    r = run("--help")
    assert r.returncode == 0 and "count" in r.stdout and "compare" in r.stdout


@pytest.mark.parametrize("k", ["33", "0"])
def test_invalid_k_message(tmp_path, k):
    # count_tests.rs:290-332
    r = run("count", "-k", k, "-i", str(tmp_path / "x.fa"), "-o", str(tmp_path / "o.tsv"))
    assert r.returncode == 1
    assert f"Invalid K-mer size: {k}. Must be between 1 and 32." in r.stderr
    assert "ERROR orion_kmer] Error: " in r.stderr


def test_build_invalid_k(tmp_path):
    r = run("build", "-k", "40", "-g", str(tmp_path / "x.fa"), "-o", str(tmp_path / "o.db"))
    assert r.returncode == 1 and "Invalid K-mer size: 40. Must be between 1 and 32." in r.stderr


def test_usage_errors_exit_2(tmp_path):
    assert run("count", "-k", "5", "-o", "x").returncode == 2              # missing -i
    assert run("count", "-i", "a", "-o", "x").returncode == 2              # missing -k
    assert run("count", "-k", "five", "-i", "a", "-o", "x").returncode == 2
    assert run("count", "-k", "300", "-i", "a", "-o", "x").returncode == 2  # not a u8
    assert run("count", "-k", "5", "-i", "a", "-o", "x", "--bogus").returncode == 2
    assert run("frobnicate").returncode == 2
    assert run().returncode == 2


def test_query_host_side_errors(tmp_path):
    # utils.rs:40-41 / :46-47 contexts (query.rs:28 loads the DB first)
    r = run("query", "-d", str(tmp_path / "missing.db"), "-r", "y", "-o", str(tmp_path / "o.txt"))
    assert r.returncode == 1 and "Failed to get input reader for k-mer database" in r.stderr
    bad = tmp_path / "bad.db"
    bad.write_bytes(b"\x04\x01")
    r = run("query", "-d", str(bad), "-r", "y", "-o", str(tmp_path / "o.txt"))
    assert r.returncode == 1 and "Failed to deserialize KmerDbV2 from" in r.stderr
    import okm
    db33 = tmp_path / "k33.db"
    okm.KmerDb(33, {"a": np.array([1, 2], np.uint64)}).write(str(db33))
    r = run("query", "-d", str(db33), "-r", "y", "-o", str(tmp_path / "o.txt"))
    assert r.returncode == 1 and "Invalid K-mer size: 33. Must be between 1 and 32." in r.stderr
    assert run("query", "-d", str(db33)).returncode == 2  # clap: missing required args


def test_classify_host_side_errors(tmp_path):
    import okm
    p4, p3 = tmp_path / "k4.db", tmp_path / "k3.db"
    okm.KmerDb(4, {"dbk4.fa": np.array([27], np.uint64)}).write(str(p4))
    okm.KmerDb(3, {"dbk3.fa": np.array([6], np.uint64)}).write(str(p3))
    out = str(tmp_path / "o.json")
    # classify_tests.rs:480-508, :510-547 — fail before the input is read
    r = run("classify", "-i", "dummy_input.fa", "-d", str(p4), "--kmer-size", "3", "-o", out)
    assert r.returncode == 1
    assert "User-provided k-mer size 3 does not match k-mer size 4 from database" in r.stderr
    r = run("classify", "-i", "dummy_input.fa", "-d", str(p4), "-d", str(p3), "-o", out)
    assert r.returncode == 1
    assert "Effective k-mer size 4 (from first database) does not match k-mer size 3 from database" in r.stderr
    r = run("classify", "-i", "dummy_input.fa", "-d", str(p4), "--kmer-size", "40", "-o", out)
    assert r.returncode == 1 and "Invalid K-mer size: 40. Must be between 1 and 32." in r.stderr
    r = run("classify", "-i", "dummy_input.fa", "-d", str(tmp_path / "nope.db"), "-o", out)
    assert r.returncode == 1 and "Failed to load database:" in r.stderr
    assert "DEBUG: Entered run_classify." in r.stderr  # classify.rs:59-64
    assert not os.path.exists(out)


@pytest.mark.skipif(has_gpu(), reason="a HIP device is visible")
def test_count_without_gpu_fails_loudly(tmp_path):
    p = tmp_path / "a.fa"
    p.write_text(">a\nACGT\n")
    r = run("count", "-k", "3", "-i", str(p), "-o", str(tmp_path / "o.tsv"))
    assert r.returncode == 1 and "no CPU fallback" in r.stderr
    assert not (tmp_path / "o.tsv").exists()
