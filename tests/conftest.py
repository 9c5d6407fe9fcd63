import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")
    # A GPU test process holds two HIP runtimes: PyTorch's bundled one (tests
    # that hand torch device buffers to the async C-ABI calls) and the one
    # libmbx links from /opt/rocm.  PyTorch's has to initialise first, as in
    # bench.py; on a machine without a GPU this is a no-op.
    if "not gpu" not in (config.getoption("-m") or ""):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass


@pytest.fixture(scope="session")
def minidata():
    import helpers
    import oracle
    rows = helpers.load_minidata()
    return rows, oracle.Table(helpers.minidata_columns(rows))


@pytest.fixture
def tune(ctx):
    """ctx.set_tuning for one test (the A/B knobs; every context starts on
    the production defaults), restored to the defaults afterwards."""
    yield ctx.set_tuning
    ctx.set_tuning("reset")
