import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sample-s3-hybrid-cache_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libs3hc_lz4.so on the GPU)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O  # noqa: E402  (test infrastructure only)

    O.lib()
    return O


@pytest.fixture(scope="session")
def engine():
    import s3hc_lz4 as S

    eng = S.Engine(0)
    yield eng
    eng.close()
