"""Debug tooling: the DPA_SYNC_CHECK op proxy."""
import math

import pytest

from distributed_pipeline_amd.ops._ext import _SyncChecked


def test_sync_checked_proxy_passes_results_through():
    m = _SyncChecked(math)
    assert m.sqrt(4.0) == 2.0
    assert m.pi == math.pi          # non-function attributes are returned as is
    assert not hasattr(m, "no_such_op")


def test_sync_checked_proxy_names_the_failing_op():
    m = _SyncChecked(math)
    with pytest.raises(RuntimeError, match=r"\[DPA_SYNC_CHECK\] native op sqrt\(-1\)"):
        m.sqrt(-1)
