"""Shared pytest setup: import paths, the `gpu` marker, fixtures for goldens and the HIP library."""
import json
import os
import sys

import numpy as np
import pytest

# The GPU tests run at the box's own hardware-queue count (GPU_MAX_HW_QUEUES, 4 on the MI355X pool): shards on one
# device share one set of four streams, the library's streams use the high-priority queue pool, and every host wait
# is bounded (rr_set_timeout), so a stream that never drains fails the test naming its shard and stream.

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "rag-serving-system_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C-ABI)")
    config.addinivalue_line("markers", "big: full-size (1M-row) parity cases")


@pytest.fixture(scope="session")
def golden_data():
    return dict(np.load(os.path.join(GOLDEN, "golden_data.npz")))


@pytest.fixture(scope="session")
def golden_synth():
    return dict(np.load(os.path.join(GOLDEN, "golden_synth.npz")))


@pytest.fixture(scope="session")
def golden_configs():
    return dict(np.load(os.path.join(GOLDEN, "golden_configs.npz")))


@pytest.fixture(scope="session")
def golden_edges():
    with open(os.path.join(GOLDEN, "golden_edge_cases.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def short_facts():
    return np.load(os.path.join(GOLDEN, "data", "short_facts_embeddings.npy"))


@pytest.fixture(scope="session")
def squad():
    return np.load(os.path.join(GOLDEN, "data", "squad_embeddings.npy"))


@pytest.fixture(scope="session")
def hip():
    """The loaded C-ABI library; GPU tests fail loudly (not skip) if it is missing."""
    # torch (plumbing for the device-pointer test) ships its own libamdhip64.so.7; let it initialise the
    # runtime first so that both share one HIP runtime in this process (same SONAME).
    try:
        import torch
        torch.cuda.is_available()
    except Exception:
        pass
    from rag_service_amd import _lib
    return _lib.load_library()
