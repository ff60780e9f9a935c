"""bench.py's rank launcher (no GPU needed): `--gpus N` with no launcher around it starts N
ranks under torch.distributed.run; a world that differs from --gpus is an error."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run(args, **env):
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e,
                          capture_output=True, text=True, timeout=120)


def test_launch_cmd_starts_n_ranks():
    import bench
    cmd = bench.launch_cmd(8, ["--gpus", "8", "--steps", "3"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1" and "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]
    assert os.path.samefile(cmd[-5], os.path.join(ROOT, "bench.py"))


def test_world_mismatch_exits_nonzero():
    r = _run(["--gpus", "3", "--no-cpu-baseline"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2, r.stderr
    assert "--gpus 3 but the launcher started 2 ranks" in r.stderr


def test_too_few_gpus_for_rccl_exits_nonzero():
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    r = _run(["--gpus", str(n), "--no-cpu-baseline"], MMDX_DIST_BACKEND="nccl")
    assert r.returncode == 2, r.stderr
    assert f"--gpus {n} needs {n} GPUs for RCCL" in r.stderr


def test_gpus_must_be_positive():
    r = _run(["--gpus", "0"])
    assert r.returncode != 0 and "--gpus must be >= 1" in r.stderr
