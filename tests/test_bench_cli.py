"""bench.py's process contract, on CPU: --gpus N drives N rank processes (it
starts torchrun itself when no WORLD_SIZE is set, before touching a GPU), and
refuses a WORLD_SIZE that disagrees with --gpus."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_world_size_mismatch_is_an_error():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_gpus_n_spawns_n_ranks(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    seen = {}

    class R:
        returncode = 0

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return R()

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    args = bench.parse()
    assert bench.launch_ranks(args) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def test_verify_sample_hits_every_lane_position():
    sys.path.insert(0, ROOT)
    import numpy as np
    import bench
    from mirbft_amd import workloads as W
    from oracle import oracle
    w = W.c2_requests(n=65536)
    out = oracle.openssl_digest_batch(w.arena, w.off, w.len, 4)
    bench.verify_sample(w, out)                     # passes on correct digests
    bad = out.copy()
    bad[65535, 0] ^= 1                              # the last digest is always sampled
    with pytest.raises(SystemExit):
        bench.verify_sample(w, bad)


def test_host_api_leg_failure_is_reported_not_fatal(monkeypatch):
    """The host_api leg runs `bench.py --mode lib` as a child after the headline
    is timed; when the child fails (here: no GPU, so no context) the leg returns
    an error object instead of raising, so the headline line is still printed.
    The torchrun variables are not passed on (the child is one process over all
    the job's GPUs), and --share-device maps the ranks onto virtual shards."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--share-device"])
    args = bench.parse()
    seen = {}
    real_run = subprocess.run

    def spy(cmd, *a, **k):
        seen["cmd"], seen["env"] = cmd, k.get("env", {})
        return real_run(cmd + ["--no-host-api"], *a, **k)

    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("MASTER_PORT", "29999")
    monkeypatch.setattr(subprocess, "run", spy)
    res = bench.host_api_leg(args, 2)
    assert "error" in res, res
    assert seen["cmd"][2:] == ["--mode", "lib", "--config", "c5", "--gpus", "1", "--steps", "5", "--warmup", "2"]
    assert "WORLD_SIZE" not in seen["env"] and "MASTER_PORT" not in seen["env"]
    assert seen["env"]["MSHA_VIRTUAL_SHARDS"] == "2"


def test_c5_forms_share_the_workload_and_count_hashed_blocks():
    """The three c5 forms build the same storm slice; only c5_folded's hashed
    blocks (its roofline numerator) drop: each distinct (off, len) once."""
    sys.path.insert(0, ROOT)
    import bench
    import numpy as np
    assert set(bench.C5_FORMS) == set(bench.C5_FORM_NOTES)
    w = bench.build_workload("c5_folded", 3, 64)        # 2^17 actions of the node's storm
    w2 = bench.build_workload("c5", 3, 64)
    assert np.array_equal(w.off, w2.off) and np.array_equal(w.len, w2.len)
    assert bench.hashed_blocks(w, "c5") == bench.hashed_blocks(w, "c5_planned") == w.blocks
    key = np.unique(np.stack([w.off, w.len], axis=1), axis=0)
    L = key[:, 1]
    exp = int(((L >> np.uint64(6)) + np.where((L & np.uint64(63)) < 56, 1, 2).astype(np.uint64)).sum())
    assert bench.hashed_blocks(w, "c5_folded") == exp < w.blocks
