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
    """The raster parity tests' element-wise strict rates (tests/parity_report.py): written to
    gpurun_out/parity_rates.txt on every run, and printed at the end of the run only when
    nothing failed -- a ~16 KB table printed after a failure pushes the failure's assertion
    text out of the tail a driver keeps."""
    try:
        from tests import parity_report
    except Exception:
        return
    if parity_report.RECORDS:
        table = parity_report.table()
        try:
            os.makedirs("gpurun_out", exist_ok=True)
            with open(os.path.join("gpurun_out", "parity_rates.txt"), "w") as f:
                f.write(table + "\n")
        except OSError:
            pass
        if exitstatus == 0:
            terminalreporter.write_sep("=", "raster parity: strict rates")
            terminalreporter.write_line(table)
        else:
            terminalreporter.write_line("raster parity strict rates: gpurun_out/parity_rates.txt")
