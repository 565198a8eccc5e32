import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "fullsize: parity at the bench's full BASELINE sizes (minutes, ~12 GB host RAM)")


@pytest.fixture(scope="session")
def built():
    import __graft_entry__ as g
    g.build()
    return True
