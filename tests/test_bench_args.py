"""bench.py's launch-mode resolution (CPU): --gpus N never silently measures fewer GPUs."""
import os
import subprocess
import sys

import pytest

import bench


def visible(n):
    return lambda: n


def test_single_default():
    assert bench.resolve_mode(1, 1, -1, visible(0)) == "single"


def test_group_when_no_launcher():
    assert bench.resolve_mode(4, 1, -1, visible(8)) == "group"
    assert bench.resolve_mode(1, 1, 1, visible(1)) == "group"      # --group 1 at N = 1


def test_torchrun_when_launched():
    assert bench.resolve_mode(8, 8, -1, visible(0)) == "torchrun"
    assert bench.resolve_mode(1, 2, -1, visible(0)) == "torchrun"


@pytest.mark.parametrize("gpus,world,group,vis", [(4, 1, -1, 2), (2, 1, 1, 1), (2, 1, 0, 8), (4, 2, -1, 8),
                                                  (1, 1, 1, 0)])
def test_refusals(gpus, world, group, vis, capsys):
    with pytest.raises(SystemExit) as e:
        bench.resolve_mode(gpus, world, group, visible(vis))
    assert e.value.code == 2
    assert "bench.py:" in capsys.readouterr().err


def test_cli_refuses_without_devices(root):
    # no GPU in this container: `--gpus 2` must exit non-zero with the reason, not report one GPU
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--cpu-baseline", "0"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 2, (r.returncode, r.stdout, r.stderr)
    assert "visible" in r.stderr
    assert r.stdout.strip() == ""
