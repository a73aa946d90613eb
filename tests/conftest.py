"""Shared test setup: import paths, the `gpu` marker, fixture loaders."""
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "rigidbody-rs_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def load_npz(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def _strict_constant(c):
    raise ValueError(f"non-strict JSON constant {c}")


def run_bench(args, env=None, timeout=300):
    """`python bench.py <args>` as the driver runs it: returns (the one stdout line, strict-parsed;
    the full detail file bench.py writes beside it).  Asserts exactly one stdout line, strict JSON
    (no NaN / Infinity tokens) and under 16 KB."""
    import subprocess
    import tempfile

    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    e["RB_BENCH_DETAIL"] = os.path.join(tempfile.mkdtemp(), "detail.json")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=e)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    assert len(lines[0]) < 16384, len(lines[0])
    line = json.loads(lines[0], parse_constant=_strict_constant)
    with open(e["RB_BENCH_DETAIL"]) as f:
        full = json.load(f, parse_constant=_strict_constant)
    return line, full


@pytest.fixture(scope="session")
def fr3_text():
    from rigidbody_amd import chains

    return chains.fr3_urdf_text()


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle

    oracle.build()
    return oracle
