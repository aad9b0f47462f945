"""The driver's round-end smoke check (__graft_entry__.smoke) as a GPU test, so the suite covers it."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.mark.gpu
def test_entry_smoke(capsys):
    import __graft_entry__ as entry
    entry.smoke()
    assert "smoke ok" in capsys.readouterr().out
