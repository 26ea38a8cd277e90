import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "consensus-specs_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    import json
    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "bls_vectors.json")) as f:
        vec = json.load(f)
    with open(os.path.join(d, "bls_golden_batches.json")) as f:
        gb = json.load(f)
    return vec, gb


@pytest.fixture(scope="session")
def native():
    """The HIP engine; GPU tests fail loudly if it is not loadable.

    Some GPU tests hand torch-allocated device buffers to the engine.  The torch
    wheel bundles its own HIP runtime: it has to be loaded before the engine's
    (bench.py imports torch first too), so that both use one runtime."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    from bls381_amd import _native
    _native.init(0)
    return _native


@pytest.fixture(scope="session")
def noncanon():
    """tests/golden/bls_noncanonical.json (make_noncanonical_vectors.py): encodings py_ecc
    1.7.0's lax codec reads and the spec's strict codec rejects, with both columns."""
    import json
    with open(os.path.join(ROOT, "tests", "golden", "bls_noncanonical.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def torsion(noncanon):
    """The cases on which the two policies may differ, with py_ecc and spec-strict verdict
    columns: tests/golden/bls_torsion.json (make_torsion_vectors.py: points outside G1/G2)
    with the verify / verify_multiple cases of bls_noncanonical.json appended, so every
    layout test that runs the torsion cases runs the non-canonical encodings too.  The
    aggregate lists are bls_torsion.json's (bls_noncanonical.json's have two output columns)."""
    import json
    with open(os.path.join(ROOT, "tests", "golden", "bls_torsion.json")) as f:
        t = json.load(f)
    t["verify"] = t["verify"] + noncanon["verify"]
    t["verify_multiple"] = t["verify_multiple"] + noncanon["verify_multiple"]
    return t
