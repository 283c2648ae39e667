"""The orion-kmer CLI's host-side contract (cli.rs / main.rs): flags, usage
errors (exit 2), the reference's error strings (exit 1), no GPU needed."""

import subprocess

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


def test_out_of_scope_subcommands_are_explicit():
    r = run("query", "-d", "x", "-r", "y", "-o", "z")
    assert r.returncode == 1 and "outside this engine's scope" in r.stderr


@pytest.mark.skipif(has_gpu(), reason="a HIP device is visible")
def test_count_without_gpu_fails_loudly(tmp_path):
    p = tmp_path / "a.fa"
    p.write_text(">a\nACGT\n")
    r = run("count", "-k", "3", "-i", str(p), "-o", str(tmp_path / "o.tsv"))
    assert r.returncode == 1 and "no CPU fallback" in r.stderr
    assert not (tmp_path / "o.tsv").exists()
