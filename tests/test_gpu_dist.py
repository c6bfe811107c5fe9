"""GPU: bench.py's N > 1 path on the HIP engine.  Two ranks (gloo, both on
cuda:0 -- the box has one GPU; on an 8-GPU node the driver runs the same code
with RCCL, one rank per GPU) launched by torch.distributed.run as a fresh
child process (and one rank over RCCL, `test_rccl_branch_one_rank`).  Config 5 is one 8M-frame job sharded by bytes: the ranks'
outputs, gathered and concatenated, must equal the reference's digest of the
whole job; config 2 is weak scaling: rank 0's batch is the digested one."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_dist(config, steps=2, extra=(), nproc=2, backend="gloo"):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
           str(nproc), "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--same-device",
           "--dist-backend", backend, "--config", str(config), "--steps", str(steps), "--warmup", "1",
           "--reps", "2", "--ramp-ms", "0", "--no-ceiling", "--no-cpu-baseline", *extra]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def run_bare(config, nproc=2, steps=2, extra=()):
    """The command the driver runs, bare: no torch.distributed.run around it,
    no WORLD_SIZE in the environment -- bench.py starts its own ranks."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--same-device",
           "--dist-backend", "gloo", "--config", str(config), "--steps", str(steps),
           "--warmup", "1", "--reps", "2", "--ramp-ms", "0", "--no-ceiling", "--no-cpu-baseline",
           *extra]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bare_command_launches_its_ranks():
    """`bench.py --gpus 2` with no launcher runs 2 ranks and
    reports them; config 5's shards concatenate to the reference's digest."""
    line = run_bare(5)
    assert line["n_gpus"] == 2 and line["per_rank"]["ranks"] == 2
    assert line["config"]["parallelism"] == "dp2"
    assert line["config"]["frames_total"] == 8 << 20
    assert line["parity_digest"]["ok"] is True, line["parity_digest"]
    assert "concatenated outputs of 2 ranks" in line["parity_digest"]["what"]


def test_shard_alone_digest():
    """`--shard 7/8`: one process times the last rank's share of the 8-GPU
    job alone; its output equals the reference's digest of that shard."""
    line = run_bare(5, nproc=1, extra=("--shard", "7/8"))
    assert line["n_gpus"] == 1 and line["config"]["shard"].startswith("7/8")
    assert line["parity_digest"]["ok"] is True, line["parity_digest"]
    assert "sha256_out_shards8[7]" in line["parity_digest"]["what"]
    assert line["parity_spot_check"] is True


def test_two_ranks_config5_sharded_digest():
    line = run_dist(5)
    assert line["n_gpus"] == 2 and line["config"]["frames_total"] == 8 << 20
    assert line["parity_digest"]["ok"] is True, line["parity_digest"]
    assert "concatenated outputs of 2 ranks" in line["parity_digest"]["what"]
    assert line["parity_spot_check"] is True


def test_two_ranks_config2_weak_scaling():
    line = run_dist(2, steps=4)
    assert line["n_gpus"] == 2 and line["config"]["frames_total"] == 2 << 20
    assert line["scaling"] == "weak"
    assert line["parity_digest"]["ok"] is True
    check_per_rank(line, 2)


def check_per_rank(line, world):
    """Every rank's kernel time and rate reach rank 0's line; the roofline
    fraction comes from the slowest rank (an 8-GPU run shows a slow GPU)."""
    pr = line["per_rank"]
    assert pr["ranks"] == world and len(pr["kernel_ms"]) == world
    assert len(pr["achieved_GBps"]) == world and all(v > 0 for v in pr["achieved_GBps"])
    lo, med, hi = pr["kernel_ms_min_median_max"]
    assert lo <= med <= hi == max(pr["kernel_ms"])
    slow = pr["kernel_ms"].index(hi)
    assert abs(line["roofline"]["achieved"] - pr["achieved_GBps"][slow]) <= 0.2
    assert line["parity_ok"] is True and line["value"] is not None


def test_two_ranks_config5_per_rank_fields():
    line = run_dist(5)
    check_per_rank(line, 2)


@pytest.mark.parametrize("config", [2, 5])
def test_rccl_branch_one_rank(config):
    """The RCCL branch on the box's one GPU: a one-rank `nccl` process group
    (--dist-init) runs the barrier, the MAX/SUM reductions, the per-rank
    all_gather and, for config 5, the shard gather, all on device tensors,
    as every rank of the driver's 8-GPU run does (two ranks cannot share one
    GPU under RCCL)."""
    line = run_dist(config, steps=2, extra=("--dist-init",), nproc=1, backend="nccl")
    assert line["n_gpus"] == 1
    assert line["parity_digest"]["ok"] is True, line["parity_digest"]
    if config == 5:
        assert "concatenated outputs of 1 ranks" in line["parity_digest"]["what"]
    check_per_rank(line, 1)
