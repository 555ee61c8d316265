"""Shared pytest configuration.

Markers: ``gpu`` — needs a real MI355X (HIP device) and the built libtfidf.so.
CPU-only tests (``-m "not gpu"``) cover the oracle against the golden vectors,
the host logic, the C-ABI library's exported symbols and the multi-rank
orchestration over gloo.
"""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "tf-idf-distributed-system_amd")
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")

# The library reads its TFIDF_* test knobs (forced paths, small batches, weak
# hashes) only while TFIDF_DEBUG is set; the tests set knobs per case.
os.environ.setdefault("TFIDF_DEBUG", "1")

# One HIP runtime per process: PyTorch bundles its own libamdhip64 /
# libhsa-runtime64 (same soname as /opt/rocm's).  Loaded first, it is the one
# libtfidf binds to; loaded after libtfidf it is a second runtime that finds no
# GPU ("No HIP GPUs are available").  Tests mix both, so torch goes first.
try:
    import torch  # noqa: F401
except Exception:
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an MI355X GPU and the HIP extension")


@pytest.fixture(scope="session")
def lucene_fixture():
    with open(os.path.join(GOLDEN, "lucene_sample8.json")) as f:
        return json.load(f)


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
