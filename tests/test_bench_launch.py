"""bench.py --gpus N (CPU, no GPU): without a launcher it starts N rank processes itself
through torch.distributed.run; under a launcher a world size that disagrees with --gpus
exits non-zero before anything touches torch or the GPU."""
import os
import subprocess
import sys
from pathlib import Path
from types import SimpleNamespace

ROOT = Path(__file__).resolve().parents[1]


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], env=e, capture_output=True,
                          text=True, timeout=60)


def test_world_size_mismatch_exits_nonzero():
    r = _run(["--gpus", "2"], WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr


def test_gpus_one_under_a_two_rank_launcher_exits_nonzero():
    r = _run(["--gpus", "1"], WORLD_SIZE="2", RANK="1", LOCAL_RANK="1")
    assert r.returncode == 2


def test_zero_gpus_refused():
    assert _run(["--gpus", "0"]).returncode == 2


def test_self_launch_starts_n_ranks(monkeypatch):
    import bench
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "call", fake_call)
    args = SimpleNamespace(gpus=4)
    rc = bench.launch_ranks(args, ["--gpus", "4", "--steps", "3"])
    assert rc == 7   # the children's exit code is the bench's
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-3:] == ["--gpus", "4", "--steps", "3"][-3:] and cmd[-4] == "--gpus"
    assert Path(cmd[cmd.index("--master-addr=127.0.0.1") + 2]).name == "bench.py"
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_single_gpu_and_matching_launcher_run_in_process(monkeypatch):
    import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.launch_ranks(SimpleNamespace(gpus=1), []) is None
    monkeypatch.setenv("WORLD_SIZE", "8")
    assert bench.launch_ranks(SimpleNamespace(gpus=8), []) is None
