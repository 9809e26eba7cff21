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
    a = bench.resolve(bench.parse(), 2)
    assert a.mode == "ddp" and a.gpus == 2 and a.no_secondary


@pytest.mark.parametrize("argv,world,expect", [
    ([], 1, dict(config="c2", gs="3d", anchors=0, sh_degree=None, mode="chunk")),
    ([], 8, dict(config="c2", gs="3d", anchors=0, mode="ddp")),
    (["--config", "c4"], 1, dict(gs="3d", anchors=500_000, sh_degree=2, view_dim=0, mode="chunk")),
    (["--config", "c4"], 8, dict(mode="chunk")),
    (["--config", "c5"], 4, dict(anchors=1_000_000, sh_degree=None, view_dim=3, mode="ddp")),
    (["--gs", "2d"], 1, dict(config="c3", gs="2d", anchors=0)),
    (["--anchors", "1000"], 1, dict(config="c2-anchors", anchors=1000, view_dim=3)),
    (["--config", "c5", "--mode", "chunk"], 2, dict(mode="chunk")),
])
def test_configs_resolve(bench, argv, world, expect):
    """--config fills the workload of BASELINE configs c2-c5 (c4: SH2 chunk, view_dim 0, no
    collectives; c5: 1M anchors, DDP); the c2 headline trains one scene DDP over views at N > 1."""
    a = bench.resolve(bench.parse(argv), world)
    for k, v in expect.items():
        assert getattr(a, k) == v, (k, getattr(a, k), v)


def test_secondary_lines_per_world(bench):
    a = bench.resolve(bench.parse([]), 1)
    assert bench.secondary_names(a, 1) == ["c2-fixed", "c2-anchors", "c3", "c4", "c5"]
    assert a.cameras == 16 and bench.resolve(bench.parse(["--config", "c2-fixed"]), 1).cameras == 1
    assert bench.secondary_names(bench.resolve(bench.parse([]), 8), 8) == ["c2-chunks", "c4", "c5"]
    # c2 at N > 1: the headline is DDP over views, the per-chunk mapping of the same workload a secondary
    assert bench.resolve(bench.parse([]), 8).mode == "ddp"
    assert bench.resolve(bench.parse(["--config", "c2-chunks"]), 8).mode == "chunk"
    assert "c4" not in bench.secondary_names(bench.resolve(bench.parse(["--config", "c4"]), 2), 2)


def test_camera_set_views():
    """The bench's training cameras (reference train.py:133-148 picks one per iteration): view 0
    is the scene's identity camera, the others valid rigid transforms looking at the scene
    centre, seeded (the same set on every rank and run)."""
    import torch
    from horizongs_amd.synthetic import camera_set
    cams = camera_set(16)
    assert cams.shape == (16, 4, 4) and torch.equal(cams[0], torch.eye(4))
    assert torch.equal(cams, camera_set(16))
    R = cams[:, :3, :3].double()
    assert torch.allclose(R @ R.transpose(1, 2), torch.eye(3, dtype=torch.float64).expand(16, 3, 3), atol=1e-6)
    assert torch.allclose(torch.linalg.det(R), torch.ones(16, dtype=torch.float64), atol=1e-6)
    centre = torch.tensor([0.0, 0.0, 6.0, 1.0])
    zc = (cams @ centre)[:, 2]  # the scene centre lies straight ahead of every camera
    assert torch.all(zc > 2.5) and len({round(float(z), 3) for z in zc}) > 8
