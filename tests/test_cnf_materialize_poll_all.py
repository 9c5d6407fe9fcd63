"""k_cnf_select's every-predecessor look-back (the form tables of >= 2^32
rows take, where the chained look-back's 32-bit inclusive prefixes would
overflow), forced on a context of its own by the select_dbg knob
(mbx_set_tuning "select_dbg" 128 on that context): the same numpy / two-call checks as
tests/test_cnf_materialize.py (R/index/ColumnarIndexScan.java:130-181,
:287-308)."""
import pytest

import mbx_pkg
import test_cnf_materialize as base

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m():
    return mbx_pkg.load()


@pytest.fixture(scope="module")
def ctx(m):
    c = m.Context(0)
    c.set_tuning("select_dbg", 128)
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
