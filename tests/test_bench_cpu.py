"""bench.py's launch logic on the CPU (no GPU is touched: both paths end
before bench.py imports torch).

* `--gpus N` without a launcher hands over to torch.distributed.run with N
  ranks (the child command is captured, not run);
* a launcher whose WORLD_SIZE differs from --gpus is refused (exit 2).
"""
import importlib.util
import os
import subprocess
import sys

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_gpus_n_without_launcher_starts_n_ranks(monkeypatch):
    bench = _bench()
    seen = {}

    def fake_call(cmd, env=None, cwd=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3"])
    try:
        bench.main()
    except SystemExit as e:
        assert e.code == 7  # the child's status is bench.py's status
    else:
        raise AssertionError("main() returned instead of exiting with the child's status")
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]
    assert cmd[-5].endswith("bench.py")


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr
