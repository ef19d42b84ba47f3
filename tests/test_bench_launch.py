"""bench.py's multi-rank launch (CPU): `--gpus N` without a launcher starts N rank
processes (torch.distributed.run on 127.0.0.1) before any GPU call and relays rank 0's
JSON line; under a launcher WORLD_SIZE must equal --gpus."""
import json
import os
import subprocess
import sys

import pytest

import bench

RANK_SCRIPT = r'''
import json, os, sys
import torch.distributed as dist
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
dist.barrier()
print("rank %d banner" % r)
if r == 0:
    print(json.dumps({"n_gpus": w, "argv": sys.argv[1:], "env_world": os.environ["WORLD_SIZE"]}))
dist.destroy_process_group()
'''


def test_launch_command_for_two_gpus():
    cmd = bench.launch_command(2, ["--gpus", "2", "--steps", "5"], 29999)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "2"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29999"
    assert cmd[-4:] == ["--gpus", "2", "--steps", "5"]
    assert cmd[-5] == os.path.abspath(bench.__file__)


def test_world_check():
    assert bench.world_check(1, {}) == (1, False)           # default: one GPU, no launch
    assert bench.world_check(8, {}) == (1, True)            # --gpus 8 alone: start 8 ranks
    assert bench.world_check(4, {"WORLD_SIZE": "4"}) == (4, False)
    with pytest.raises(SystemExit):                           # the launcher's world and --gpus disagree
        bench.world_check(8, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.world_check(1, {"WORLD_SIZE": "2"})


def test_relay_two_ranks(tmp_path):
    """The relay runs the ranks through torch.distributed.run and passes rank 0's JSON line on."""
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    out = tmp_path / "out.txt"
    code = ("import os, sys; sys.path.insert(0, %r); import bench; fd = os.open(%r, os.O_WRONLY | os.O_CREAT); "
            "sys.exit(bench.relay_ranks(2, ['--gpus', '2'], fd, script=%r))"
            % (os.path.dirname(os.path.abspath(bench.__file__)), str(out), str(script)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    lines = out.read_text().splitlines()
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["env_world"] == "2" and d["argv"] == ["--gpus", "2"]
