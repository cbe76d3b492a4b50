"""bench.py's multi-rank launch: `python bench.py --gpus N` without a
launcher starts N rank processes itself, and a WORLD_SIZE that disagrees with --gpus is an
error, never a silent one-GPU run.  CPU only: --launch-only joins a gloo process group and
reports the ranks that joined, without any GPU work."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra)
    return env


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-only", "--backend", "gloo"],
                       capture_output=True, text=True, timeout=180, env=_env())
    assert p.returncode == 0, p.stderr[-2000:]
    d = _json_line(p.stdout)
    assert d["n_gpus"] == n and d["ranks_joined"] == n


def test_world_size_mismatch_is_refused():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2"], capture_output=True, text=True, timeout=120,
                       env=_env(WORLD_SIZE="3", RANK="0"))
    assert p.returncode != 0
    assert "WORLD_SIZE=3" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_gpus_beyond_visible_devices_is_refused():
    """On a host without enough GPUs the launcher refuses instead of timing fewer ranks."""
    import torch
    have = torch.cuda.device_count()
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(have + 1)], capture_output=True, text=True,
                       timeout=120, env=_env())
    if have + 1 == 1:  # no GPU: --gpus 1 runs in-process and fails for lack of a device
        assert p.returncode != 0
        return
    assert p.returncode == 2
    assert "GPU(s) visible" in p.stderr
