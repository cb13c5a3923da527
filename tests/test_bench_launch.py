"""bench.py's multi-GPU entry: --gpus N > 1 without torchrun starts one rank
per GPU as a child torch.distributed.run, refuses to measure on fewer visible GPUs, and a
torchrun launch must agree with --gpus.  CPU only: the launch command is checked through
--dry-launch, and this container has no GPU, so --gpus 2 must fail before running anything."""
import json
import os
import subprocess
import sys

import pytest

from helpers import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=300, env=env)


@pytest.mark.parametrize("mode", ["chains", "sharded"])
def test_dry_launch_command(mode):
    r = _run(["--gpus", "4", "--mode", mode, "--steps", "20", "--warmup", "5", "--dry-launch"])
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    cmd = out["launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    i = cmd.index(BENCH)
    # the ranks get the same arguments, without the dry-launch flag
    assert cmd[i + 1:] == ["--gpus", "4", "--mode", mode, "--steps", "20", "--warmup", "5"]
    assert out["nproc_per_node"] == 4 and out["mode"] == mode


def test_fewer_visible_gpus_fails_loudly():
    r = _run(["--gpus", "2", "--steps", "5", "--warmup", "1"])
    assert r.returncode != 0
    assert "visible" in r.stderr and r.stdout.strip() == ""


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_roofline_evidence_is_the_newest_profile():
    sys.path.insert(0, ROOT)
    import bench
    p = bench.newest_profile("pmc.json")
    assert os.path.exists(p), p
    names = [f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("_pmc.json")]
    import re
    keys = [(int(m[1]), int(m[2])) for f in names for m in [re.fullmatch(r"r(\d+)_s(\d+)_pmc\.json", f)] if m]
    m = re.search(r"r(\d+)_s(\d+)_pmc\.json$", p)
    assert (int(m[1]), int(m[2])) == max(keys)
    t = bench.traced_launch(bench.newest_profile("kernel_stats.csv"), "z")
    assert t is not None and t["avg_us"] > 0
