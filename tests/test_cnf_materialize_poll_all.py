"""k_cnf_select's every-predecessor look-back (the form tables of >= 2^32
rows take, where the chained look-back's 32-bit inclusive prefixes would
overflow), forced on a context of its own by the select_dbg knob
(MBX_SELECT_DBG=128, read at mbx_init): the same numpy / two-call checks as
tests/test_cnf_materialize.py (R/index/ColumnarIndexScan.java:130-181,
:287-308)."""
import os

import pytest

import mbx_pkg
import test_cnf_materialize as base

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m():
    return mbx_pkg.load()


@pytest.fixture(scope="module")
def ctx(m):
    old = os.environ.get("MBX_SELECT_DBG")
    os.environ["MBX_SELECT_DBG"] = "128"
    try:
        c = m.Context(0)
    finally:
        if old is None:
            os.environ.pop("MBX_SELECT_DBG")
        else:
            os.environ["MBX_SELECT_DBG"] = old
    yield c
    c.close()


@pytest.mark.parametrize("n", [1, 65, 70_001, 700_013])
@pytest.mark.parametrize("shape", list(base.SHAPES))
def test_poll_all_matches_numpy(ctx, n, shape):
    base.test_cnf_materialize_matches_numpy(ctx, n, shape)


@pytest.mark.parametrize("density", [0.0, 0.01, 1.0])
def test_poll_all_densities_and_deleted(ctx, density):
    base.test_cnf_materialize_densities_and_deleted(ctx, density)


def test_poll_all_repeated_and_graph_replay(ctx):
    base.test_cnf_materialize_repeated_and_graph_replay(ctx)


def test_poll_all_grid_sizes_alternate(ctx):
    base.test_cnf_materialize_grid_sizes_alternate(ctx)
