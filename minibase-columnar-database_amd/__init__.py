"""MI355X-native executor for the Minibase-Columnar scan/filter/index hot path.

Layout
  csrc/        CDNA4 HIP kernels + the C-ABI implementation (-> libmbx.so)
  host/        C++ mirror of the reference's iterator/index classes over the
               C-ABI (ColumnarFileScan, ColumnIndexScan, ColumnarIndexScan,
               CondExpr ...) and the `query` / `indexes_query` driver
  mbx.py       ctypes binding of the C-ABI (tests, bench)

The directory name carries hyphens, so import it through mbx_pkg.load()
(repository root), which registers it as the module `mbx_amd`.
"""
from . import dist  # noqa: F401
from . import mbx  # noqa: F401
from .mbx import MbxError, Context, device_count, lib  # noqa: F401
