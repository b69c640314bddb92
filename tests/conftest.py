import os
import subprocess
import sys

import numpy as np
import pytest

# torch (used by the device-pointer tests) before libgpdemod: torch ships its own HIP runtime,
# and loading it after the system one our library links makes torch see no device
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def oracle():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    import oracle as o
    return o


@pytest.fixture(scope="session")
def gpd():
    import gpdemod_loader
    gpdemod_loader.load_build().build()
    return gpdemod_loader.load()


@pytest.fixture(scope="session")
def gpu(gpd):
    if gpd.load().gpd_device_count() < 1:
        pytest.fail("GPU test selected but no HIP device is visible")
    return gpd


def rel_err(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    return np.abs(a - b) / np.maximum(np.abs(b), 1e-300)


def wrap_diff(a, b):
    """|a-b| modulo 2π (ϕ compared modulo 2π after sign normalisation)."""
    d = (np.asarray(a) - np.asarray(b) + np.pi) % (2 * np.pi) - np.pi
    return np.abs(d)


@pytest.fixture
def opts(gpd):
    """opts(name, value): set one of the library's test/diagnostics options (gpd_set_option; the
    library reads no environment variable) for this test; every option is reset afterwards."""
    def set_(name, value):
        gpd.set_option(name, int(value))
    yield set_
    gpd.reset_options()
