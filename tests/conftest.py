import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device; runs the HIP kernels")


@pytest.fixture(scope="session")
def golden_dir() -> Path:
    return GOLDEN


@pytest.fixture(scope="session")
def gpu():
    """The HIP library, initialised on a gfx950 device (GPU tests only)."""
    from carbonado_amd import _lib
    L = _lib.lib()
    rc = L.chip_init(0)
    if rc != 0:
        pytest.fail(f"no usable gfx950 device: status {rc} ({L.chip_last_device_error().decode()})")
    return L
