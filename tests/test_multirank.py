"""Multi-rank sharding on CPU (gloo, world size 2): each rank builds its own
disjoint slice of the workload exactly as bench.py does, with no data-path
collective; together the slices equal the single-process workload."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mirbft_amd import workloads as W
    # bench.py's slicing: c2 -> first = rank * n ; c5 -> first = rank * (total // world)
    n = 4096
    c2 = W.c2_requests(n=n, first=rank * n)
    c5 = W.c5_storm(n=8192 // world, first=rank * (8192 // world))
    # the only collective: the harness max-reduce of elapsed time (here a dummy value)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put((rank, c2.arena[: n * 512].tobytes(), c5.len.copy(), float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_slices_cover_the_global_workload():
    import torch.multiprocessing as mp
    from mirbft_amd import workloads as W
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g2 = W.c2_requests(n=8192, first=0)
    assert res[0][1] + res[1][1] == g2.arena[: 8192 * 512].tobytes()
    g5 = W.c5_storm(n=8192, first=0)
    assert np.array_equal(np.concatenate([res[0][2], res[1][2]]), g5.len)
    assert res[0][3] == res[1][3] == 2.0   # max over ranks


def test_partition_matches_rank_slicing_balance():
    from mirbft_amd.engine import partition_by_blocks, blocks_for_len
    from mirbft_amd import workloads as W
    w = W.c5_storm(n=1 << 14)
    b = partition_by_blocks(w.len, 8)
    blocks = np.array([blocks_for_len(int(x)) for x in w.len])
    per = np.array([blocks[b[i]:b[i + 1]].sum() for i in range(8)])
    assert per.sum() == blocks.sum()
    assert per.max() - per.min() <= blocks.max()


@pytest.mark.gpu
def test_bench_two_ranks_on_the_engine():
    """bench.py --gpus 2 starts its own two rank processes (no torchrun
    environment given) and each drives the HIP engine on its own disjoint c2
    slice; on a one-GPU box both ranks share GPU 0 (--share-device). Rank 0's
    stdout is exactly one JSON line with n_gpus 2 and the whole job's work."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-device",
                        "--steps", "5", "--warmup", "2", "--min-warmup-ms", "50", "--cpu-seconds", "1.5",
                        "--no-host-api-unaliased"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    # c2 runs the lane kernel (a forced MSHA_LOAD_MODE=3 A/B run makes it the pipelined one)
    want = "pipe" if os.environ.get("MSHA_LOAD_MODE") == "3" else "lane"
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["kernel"] == want
    assert "error" not in d["host_api"] and d["host_api"]["shards"] == 2
    assert d["value"] > 0 and d["config"]["messages_per_gpu"] == 1 << 20
    # BASELINE config 5 as quoted: the 2^23 storm over both ranks, kernel-resident, verified
    c5 = d["extra_configs"]["c5"]
    assert c5["n_gpus"] == 2 and c5["scaling"] == "strong" and c5["value"] > 0 and 0 < c5["frac"] < 1
    assert c5["blocks"] > 0 and "512 digests per rank" in c5["verified"]
    # ... and its GPU-planned forms (every action hashed; aliases folded)
    for form in ("c5_planned", "c5_folded"):
        f = d["extra_configs"][form]
        assert f["n_gpus"] == 2 and f["scaling"] == "strong" and f["value"] > 0 and f["blocks"] == c5["blocks"]
        assert "512 digests per rank" in f["verified"]
        # unfolded: the cooperative head; folded: the work-stealing lane kernel, the late head on the
        # two-lane chain, the early one on eight
        assert f["kernel"] == {"c5_planned": "lane+coop", "c5_folded": "lane_ws+chain2+chain8"}[form], f["kernel"]
    assert d["extra_configs"]["c5_folded"]["hashed_blocks"] < c5["blocks"] == d["extra_configs"]["c5_planned"]["hashed_blocks"]
    # the CPU baseline at N > 1 too (rank 0, after the ranks released their GPUs)
    cb = d["cpu_baseline"]
    # value = OpenSSL SHA-NI on one thread (the kind says so); the scalar port beside it
    assert cb["kind"] == "openssl-sha-ni-1-thread (proxy for Go crypto/sha256)"
    assert cb["cores"] == 1 and cb["value"] == cb["openssl"]["1_thread"]["value"] and cb["impl"]
    assert cb["scalar_port"]["value"] > 0
    assert d["host_api"]["first_launch_ms_max"] > 0


def _summary_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    out = {}
    for form in bench.C5_FORMS:
        # each rank's own figures, as extra_c5_ranks measures them on its GPU
        out[form] = bench.c5_rank_summary(dist, world, form, n=1 << 20, nbytes=1 << 29, blocks=47_000_000 + rank,
                                          hashed=8_000_000, max_blocks=1427 - rank, elapsed=0.02 + rank * 1e-3,
                                          kern_ms=2.0 + rank * 0.01, clock_ghz=2.3, steps=10)
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def test_eight_rank_c5_line_reports_each_rank():
    """a default bench line over 8 ranks (the driver's 8-GPU node)
    carries, for c5_planned and c5_folded, every rank's kernel time, its longest
    payload and the chain head's estimated share -- faked here with 8 gloo ranks on
    the CPU (bench.c5_rank_summary is what extra_c5_ranks reports); and host_api
    carries each GPU's upload rate (bench.host_api_summary)."""
    import torch.multiprocessing as mp
    import bench
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_summary_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for form in bench.C5_FORMS:
        e = out[form]
        assert e["n_gpus"] == world and len(e["kernel_ms_per_rank"]) == world
        assert e["kernel_ms_per_rank"] == [2.0 + r * 0.01 for r in range(world)]
        assert e["kernel_ms_mean_max_over_ranks"] == max(e["kernel_ms_per_rank"])
        assert e["max_blocks_per_rank"] == [1427 - r for r in range(world)]
        assert e["blocks"] == sum(47_000_000 + r for r in range(world))
        if form == "c5":
            assert "head_share_est_per_rank" not in e
        else:
            est = e["head_chain_ms_est_per_rank"]
            assert len(est) == world and abs(est[0] - 1427 * bench.HEAD_CYCLES_PER_BLOCK[form] / 2.3e6) < 1e-9
            assert all(0 < s < 2 for s in e["head_share_est_per_rank"])
    # host_api: per-GPU upload GB/s from a --mode lib line over 8 GPUs
    shards = [{"device": g, "messages": 1 << 20, "lanes": 1 << 20, "head_lanes": 12, "h2d_bytes": 480e6,
               "device_ms": 10.0, "upload_ms": 8.0 + g, "kernel_ms": 2.0, "first_launch_ms": 1.5,
               "plan_kernel_ms": 0.2} for g in range(world)]
    d = {"arena_bytes": 1, "value": 8e8, "n_gpus": world, "shards": world, "virtual_shards": None,
         "ms_per_step": 11.0, "call_ms": [11.0], "gbps_hashed": 300.0, "steps": 5,
         "last_call_stats": {"plan_ms": 1.5}, "last_call_shards": shards}
    h = bench.host_api_summary(d, "test")
    assert [g["upload_gbps"] for g in h["per_gpu"]] == [480e6 / (8.0 + g) / 1e6 for g in range(world)]
    assert h["upload_gbps_min"] == 480e6 / 15.0 / 1e6 and h["upload_gbps_max"] == 60.0
