"""CPU tests of bench.py's multi-GPU launcher: `--gpus N` without WORLD_SIZE starts N ranks
through torch.distributed.run in a child process (never an exec, nothing touches the GPU in
the parent); under torchrun (WORLD_SIZE set) or for N = 1 it does nothing."""
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # __name__ != "__main__": neither the launcher nor main() runs
    return mod


def _run(bench, monkeypatch, argv, env_world=None):
    calls = []
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    if env_world is None:
        monkeypatch.delenv("WORLD_SIZE", raising=False)
    else:
        monkeypatch.setenv("WORLD_SIZE", env_world)
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: calls.append((cmd, env)) or 0)
    try:
        bench._launch_ranks()
        code = None
    except SystemExit as e:
        code = e.code
    return calls, code


def test_launcher_starts_n_ranks(bench, monkeypatch):
    calls, code = _run(bench, monkeypatch, ["--gpus", "4", "--steps", "7", "--warmup", "2"])
    assert code == 0 and len(calls) == 1
    cmd, env = calls[0]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[cmd.index(os.path.join(ROOT, "bench.py")) + 1:] == ["--gpus", "4", "--steps", "7", "--warmup", "2"]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_launcher_equals_form_and_exit_code(bench, monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus=2"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: 3)
    with pytest.raises(SystemExit) as e:
        bench._launch_ranks()
    assert e.value.code == 3  # the children's status is the parent's


@pytest.mark.parametrize("argv,world", [(["--gpus", "1"], None), ([], None), (["--gpus", "8"], "8")])
def test_launcher_noop(bench, monkeypatch, argv, world):
    calls, code = _run(bench, monkeypatch, argv, env_world=world)
    assert calls == [] and code is None


def test_parser_has_modes(bench, monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--mode", "ddp", "--gpus", "2", "--no-secondary"])
    a = bench.parse()
    assert a.mode == "ddp" and a.gpus == 2 and a.no_secondary
