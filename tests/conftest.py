import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AMD = os.path.join(ROOT, "orion-kmer_amd")
for p in (ROOT, AMD, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) HIP device; parity tests proper")
    config.addinivalue_line("markers", "slow: multi-second CPU test")


def _ensure_built():
    lib = os.path.join(AMD, "build", "liborion_kmer.so")
    cli = os.path.join(AMD, "build", "orion-kmer")
    if not (os.path.exists(lib) and os.path.exists(cli)):
        subprocess.run(["make", "-s", "-C", AMD, "-j8"], check=True)
    olib = os.path.join(ROOT, "oracle", "build", "liboracle.so")
    if not os.path.exists(olib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


@pytest.fixture(scope="session", autouse=True)
def built_libraries():
    _ensure_built()
    yield


@pytest.fixture(autouse=True)
def _reset_test_knobs():
    """Every engine test hook (okm.testing) back to its product default after
    each test, whatever the test set."""
    yield
    try:
        from okm import testing
        testing.reset_all()
    except Exception:  # no library (a pure-Python test on a bare checkout)
        pass


@pytest.fixture(scope="session")
def golden_cases():
    import json
    with open(os.path.join(GOLDEN, "cases.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def reference_expectations():
    import json
    with open(os.path.join(GOLDEN, "reference_expectations.json")) as fh:
        return json.load(fh)


def case_file_bytes(f):
    if "text" in f:
        return f["text"].encode()
    with open(os.path.join(GOLDEN, "data", f["fixture"]), "rb") as fh:
        return fh.read()


def materialize(tmp_path, files, subdir="in"):
    """Write a case's input files under tmp_path; returns their paths."""
    d = tmp_path / subdir
    d.mkdir(parents=True, exist_ok=True)
    paths = []
    for f in files:
        p = d / f["name"]
        p.write_bytes(case_file_bytes(f))
        paths.append(str(p))
    return paths


def has_gpu():
    try:
        import okm
        return okm.device_count() > 0
    except Exception:
        return False
