import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")


@pytest.fixture(scope="session")
def minidata():
    import helpers
    import oracle
    rows = helpers.load_minidata()
    return rows, oracle.Table(helpers.minidata_columns(rows))
