"""CPU: bench.py's own N-rank launcher.  A bare
`python3 bench.py --gpus N` starts N rank processes itself (one per GPU,
LOCAL_RANK = GPU) before torch or any GPU call; under torch.distributed.run
it is one rank; a WORLD_SIZE that disagrees with --gpus is an error.  The
launch itself is exercised with a stand-in rank script (no GPU here); the GPU
test runs the real bare command (tests/test_gpu_dist.py)."""
import os
import subprocess
import sys
import textwrap

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("gpus,env,plan", [
    (1, {}, "run"),
    (2, {}, "launch"),
    (8, {}, "launch"),
    (8, {"WORLD_SIZE": "8"}, "run"),          # under torch.distributed.run / launch_ranks
    (1, {"WORLD_SIZE": "1"}, "run"),
    (8, {"WORLD_SIZE": "1"}, "error"),
    (2, {"WORLD_SIZE": "4"}, "error"),
    (1, {"WORLD_SIZE": "2"}, "error"),
    (2, {"WORLD_SIZE": "x"}, "error"),
    (0, {}, "error"),
])
def test_launch_plan(gpus, env, plan):
    got, msg = bench.launch_plan(gpus, env)
    assert got == plan
    assert (msg is not None) == (plan == "error")


def test_rank_env_is_torchrun_shaped():
    env = bench.rank_env({"PATH": "/bin"}, 3, 8, 12345)
    assert env["RANK"] == env["LOCAL_RANK"] == "3"
    assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "8"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "12345"
    assert env["PATH"] == "/bin" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # a rank sees itself as "run", never launches again
    assert bench.launch_plan(8, env)[0] == "run"


RANK_SCRIPT = textwrap.dedent("""
    import os, sys, time
    r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    mode = sys.argv[1]
    if mode == "ok":
        print(f'{{"rank": {r}, "world": {w}, "local": {os.environ["LOCAL_RANK"]}, '
              f'"port": {os.environ["MASTER_PORT"]}, "argv": "{" ".join(sys.argv[1:])}"}}',
              flush=True)
        sys.exit(0)
    if mode == "fail1":
        if r == 1:
            sys.exit(7)
        time.sleep(60)        # would block in a barrier forever
""")


def _run_launcher(tmp_path, world, mode, grace):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
            f"sys.exit(bench.launch_ranks({world}, [{mode!r}, '--x'], grace_s={grace}, "
            f"script={str(script)!r}))")
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          timeout=120, cwd=ROOT)


def test_launch_ranks_rank0_stdout_only(tmp_path):
    """N rank processes with torchrun's variables; only rank 0's stdout is the
    parent's stdout (the one JSON line); the others go to stderr; rc 0."""
    import json
    r = _run_launcher(tmp_path, 4, "ok", 5)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["rank"] == 0 and lines[0]["world"] == 4
    assert lines[0]["local"] == 0 and lines[0]["argv"] == "ok --x"
    others = [json.loads(x) for x in r.stderr.splitlines() if x.startswith("{")]
    assert sorted(o["rank"] for o in others) == [1, 2, 3]
    assert len({o["port"] for o in others + lines}) == 1


def test_launch_ranks_failure_kills_the_rest(tmp_path):
    """A failing rank's code is the launcher's; the ranks left waiting are
    killed after the grace period instead of hanging the job."""
    import time
    t = time.monotonic()
    r = _run_launcher(tmp_path, 3, "fail1", 1.0)
    assert r.returncode == 7
    assert time.monotonic() - t < 30
    assert "rank 1 exited with 7" in r.stderr and "killed after rank failure" in r.stderr


def _bench(args, env_extra):
    env = dict(os.environ, **env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)


def test_bench_rejects_world_size_mismatch():
    """WORLD_SIZE != --gpus: rc 2 before anything touches a GPU."""
    r = _bench(["--gpus", "8"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2 but --gpus 8" in r.stderr


def test_bench_shard_needs_one_process():
    r = _bench(["--gpus", "2", "--shard", "0/8"], {})
    assert r.returncode == 2 and "--shard" in r.stderr
    with pytest.raises(SystemExit):
        bench.parse_shard("8/8")
    with pytest.raises(SystemExit):
        bench.parse_shard("a/b")
    assert bench.parse_shard("7/8") == (7, 8) and bench.parse_shard("") is None


def test_shard_digests_tile_the_job():
    """digests.json holds the reference's per-shard digests of config 5 for
    N = 2, 4, 8 (make_golden.py --only-shards, which checks that the shards
    concatenate to the whole-job digest)."""
    import json
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))["config5"]
    for w in (2, 4, 8):
        hs = d[f"sha256_out_shards{w}"]
        assert len(hs) == w and len(set(hs)) == w and all(len(h) == 64 for h in hs)


def test_ranks_die_with_a_killed_launcher(tmp_path):
    """A launcher killed outright (SIGKILL, as a time limit does) takes its
    rank processes with it (PR_SET_PDEATHSIG): none is left holding a GPU."""
    import signal
    import time
    script = tmp_path / "rank.py"
    script.write_text("import os, time\nprint(os.getpid(), flush=True)\ntime.sleep(120)\n")
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
            f"sys.exit(bench.launch_ranks(2, [], script={str(script)!r}))")
    p = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    pid0 = int(p.stdout.readline())           # rank 0 is up
    time.sleep(0.5)
    p.send_signal(signal.SIGKILL)
    p.wait(timeout=30)
    for _ in range(100):
        try:
            os.kill(pid0, 0)
        except ProcessLookupError:
            break
        time.sleep(0.1)
    else:
        os.kill(pid0, signal.SIGKILL)
        pytest.fail("rank 0 outlived its killed launcher")
