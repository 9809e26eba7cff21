import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.build()
    return oracle


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """The raster parity tests' element-wise strict rates (tests/parity_report.py), printed at
    the end of every run so the suite's own log carries them (also with -q)."""
    try:
        from tests import parity_report
    except Exception:
        return
    if parity_report.RECORDS:
        terminalreporter.write_sep("=", "raster parity: strict rates")
        terminalreporter.write_line(parity_report.table())
