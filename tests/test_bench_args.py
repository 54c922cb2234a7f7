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


def test_headline_is_strong_scaling_by_default():
    # the metric is "1080p 1024spp, 1/2/4/8 MI355X": the fixed C3 image at every N
    args = bench.parse_args([])
    assert args.scaling == "strong" and args.config == "C3"
    c = bench.CONFIGS[args.config]
    assert (c["width"], c["height"], c["spp"]) == (1920, 1080, 1024)


def test_gpus_below_one_exits_2(capsys):
    with pytest.raises(SystemExit) as e:
        bench.resolve_mode(0, 1, -1, visible(1))
    assert e.value.code == 2
    assert "bench.py:" in capsys.readouterr().err


def test_group_mode_timing_needs_no_torch(root):
    # --group 1: pt_group_render / pt_group_gather synchronise every device themselves, so timed()
    # brackets them without torch's barriers or events (torch may still be loaded: _native.hip()
    # imports it first to keep one HIP runtime)
    code = (
        "import sys, bench\n"
        "class R:\n"
        "    mode = 'single'\n"
        "    gather_ms = 0.0\n"
        "    def step(self): return 1.0\n"
        "e, k = bench.timed(R(), 2, 1, 0, False, use_torch=False)\n"
        "assert k == 2.0, k\n"
        "assert 'torch' not in sys.modules, 'torch imported'\n"
        "print('ok')\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=str(root), timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", (r.stdout, r.stderr)
    src = (root / "bench.py").read_text()
    # every timed() call passes the process's mode-derived flag
    assert src.count("timed(") - 1 == src.count("use_torch)")
