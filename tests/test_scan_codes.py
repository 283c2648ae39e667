"""The SWAR window helpers of okm_scan.h (shared by the extraction and query
kernels) against a per-window restatement of kmer.rs:12-106, run on the host
(the helpers are __host__ __device__).  CPU only: hipcc builds the check as a
host program."""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_scan_codes_selftest(tmp_path):
    exe = str(tmp_path / "scan_selftest")
    src = os.path.join(ROOT, "tests", "native", "scan_selftest.hip")
    inc = os.path.join(ROOT, "orion-kmer_amd", "csrc")
    subprocess.run(["/opt/rocm/bin/hipcc", "--cuda-host-only", "-O2", "-std=c++17", f"-I{inc}",
                    f"-I{os.path.join(ROOT, 'include')}", src, "-o", exe], check=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
