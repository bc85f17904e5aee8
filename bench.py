#!/usr/bin/env python3
"""Benchmark of the MI355X batched SHA-256 hash path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c3dd|c4|c5] [--mode kernel|lib]

A *step* is one pass of the hot path -- processor.ProcessHashActions
(/root/reference/pkg/processor/serial.go:180-198) over one batch of synthetic
hash actions -- with inputs already resident in HBM (kernel-resident), i.e.
one engine launch over the whole batch. Default workload: BASELINE config c2
(2^20 client requests x 512 B, request digests; the config the metric is
quoted on). N>1: one process per GPU (torchrun; started by this script itself
when WORLD_SIZE is unset), every rank hashes its own disjoint 2^20-request
slice (weak scaling, no collective on the data path); the timed region is
bracketed by barrier + synchronize and the max over ranks is taken. Rank 0
prints ONE JSON line. With --config c2 on one GPU the line also carries
extra_configs (c3, c4 and c5 timed the same way, each with its own roofline
fraction and verified sample). --mode lib instead times the north-star host
path in ONE process: one libmirsha context over N GPUs (device_mask), a pinned
arena, msha_digest_batch per step (PCIe-inclusive; never the headline value); the
default run reports it as host_api (c5 over all N GPUs, a child process). Warmup: the W steps, then more untimed
steps until --min-warmup-ms (300) of wall time has passed -- MI355X clocks need
~100 ms of load to settle, and a cold timed region measures the clock ramp
(c2: 0.395 ms per launch after 3 warmup steps, 0.330 ms after 200); the line
reports warmup_steps_run and warmup_ms.

roofline: the kernel is integer-VALU bound. achieved = 1400 int32 ops per
64-byte block (the minimal gfx950 instruction count) x blocks per
launch / mean launch time (one HIP event pair on the launch stream around the
K timed launches, divided by K: dispatch gaps included; an event pair around
every launch -- --events step -- itself cost c3 8 % per step); peak = 78.64 T
lane-ops/s (256 CU x 4 SIMD-32 x 2.4 GHz, MI355X_MICROARCH.md). cpu_baseline:
the oracle's single-threaded C restatement of the same loop on a bounded
sample, rank 0 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

OPS_PER_BLOCK = 1400           # DESIGN.md "Algorithmic work per block"
# Reference point, NOT a ceiling: the rate of the bare compression loop on
# register-resident data (no loads, no padding logic), 28.3 G blocks/s x 1400
# (tools/valu_microbench4.hip, profiles/r01_valu_microbench4.jsonl). The shipped
# c2 kernel beats it (its padding block's schedule runs on the SALU).
BARE_LOOP_TOPS = 28.3e9 * OPS_PER_BLOCK / 1e12
PEAK_VALU_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12   # 78.64 T int32 lane-ops/s
METRIC = "SHA-256 digests/sec + GB/s hashed (1/2/4/8 MI355X), % integer-ALU roofline"
# BASELINE config 5's device-resident forms: c5 = the caller's size-class order
# (msha_order_by_blocks on the host, once, as part of packing), every action
# hashed; c5_planned = msha_digest_batch_device_planned, the order planned on
# the GPU inside every timed step, longest chains on the cooperative kernel
# beside the lane kernel; c5_folded = the same with alias folding (equal
# (off, len) hashed once per step, every action still gets its digest).
C5_FORMS = ("c5", "c5_planned", "c5_folded")
C5_FORM_NOTES = {
    "c5": "caller's size-class order (host, once, part of packing); every action hashed",
    "c5_planned": "msha_digest_batch_device_planned: order planned on the GPU inside each step, longest "
                  "chains on the cooperative kernel on CUs of their own; every action hashed",
    "c5_folded": "msha_digest_batch_device_planned + MSHA_PLAN_FOLD_ALIASES: the same, equal (off, len) "
                 "hashed once per step and the digest copied to every such action (frac on hashed blocks)",
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--min-warmup-ms", type=float, default=300.0,
                   help="after the W warmup steps, keep running untimed steps until this much "
                        "wall time has passed: MI355X clocks take ~100 ms of load to settle, "
                        "and a timed region that starts cold measures the ramp, not the kernel")
    p.add_argument("--config", default="c2",
                   help="c2 (default) | c3 | c3dd (digest-of-digests form) | c4 | c5 | ub:N:SIZE (experiment: "
                        "N uniform messages via the batch kernel) | "
                        "u:N:SIZE[:STRIDE] (experiment: N uniform messages via the uniform kernel; "
                        "STRIDE 0 makes every lane hash the same cached message)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--policy", default="auto", choices=["auto", "lane", "coop"],
                   help="batch-kernel policy (msha_set_kernel_policy); digests are identical")
    p.add_argument("--events", default="span", choices=["step", "span"],
                   help="span: one HIP event pair around the K launches (default); step: a pair "
                        "around every launch (costs c3 8%% per step: the A/B of the events' cost)")
    p.add_argument("--share-device", action="store_true",
                   help="rehearsal only: every rank uses GPU 0 (multi-rank path on a 1-GPU box)")
    p.add_argument("--mode", default="kernel", choices=["kernel", "lib"],
                   help="kernel: kernel-resident, one process per GPU (the headline); lib: one process, "
                        "one libmirsha context over N GPUs (device_mask) and the host entry point "
                        "msha_digest_batch on a pinned arena (end-to-end, PCIe-inclusive)")
    p.add_argument("--pageable", action="store_true", help="with --mode lib: a pageable numpy arena")
    p.add_argument("--unaliased", action="store_true",
                   help="with --mode lib --config c5: every action packs its own copy of its payload, in "
                        "action order (a caller that does not share EpochChange payloads between actions)")
    p.add_argument("--no-extra", action="store_true",
                   help="skip the extra_configs legs (one GPU: c3, c4, c5; N GPUs: c5 over all ranks)")
    p.add_argument("--no-host-api", action="store_true",
                   help="skip the host_api legs (c5 through msha_digest_batch over all N GPUs, one process)")
    p.add_argument("--no-host-api-unaliased", action="store_true",
                   help="skip host_api_unaliased (c5 with every action its own payload copy: ~24 GB pinned)")
    return p.parse_args()


def build_workload(cfg: str, rank: int, world: int):
    from mirbft_amd import workloads as W
    if cfg == "c2":
        n = 1 << 20
        return W.c2_requests(n=n, first=rank * n)
    if cfg in ("c3", "c3dd"):
        n = 200_000
        return W.c3_batches(n=n, first=rank * n)
    if cfg == "c4":
        n = 65536
        return W.c4_large(n=n, first=rank * n)
    if cfg in C5_FORMS:
        total = 1 << 23
        per = total // world            # c5 is quoted as 8M actions over the node
        return W.c5_storm(n=per, first=rank * per)
    if cfg.startswith("ub:"):        # uniform sizes through the batch (off/len) kernel
        n, size = (int(x) for x in cfg.split(":")[1:3])
        return W.uniform_requests(n, size, W.SEED, rank * n, name=f"batch-kernel experiment {n} x {size} B")
    if cfg.startswith("u:"):
        parts = cfg.split(":")
        n, size = int(parts[1]), int(parts[2])
        w = W.uniform_requests(n, size, W.SEED, rank * n, name=f"uniform experiment {n} x {size} B")
        if len(parts) > 3:
            w.uniform_stride = int(parts[3])
        return w
    raise ValueError(cfg)


def _time_cpu(fn, n: int, nbytes_per: int, seconds: float):
    done = nbytes = 0
    t0 = time.perf_counter()
    while True:
        fn()
        done += n
        nbytes += nbytes_per
        el = time.perf_counter() - t0
        if el >= seconds:
            return done / el, nbytes / el / 1e9, done, el


CPU_THREADS = 16   # the GPU box's CPU share per GPU
# cpu_baseline.kind names what `value` timed: OpenSSL's SHA-256 (SHA-NI) on one
# thread when libcrypto loads -- a stand-in for Go's crypto/sha256, which cannot
# run here -- else the oracle's scalar C port (always reported as scalar_port).
OPENSSL_KIND = "openssl-sha-ni-1-thread (proxy for Go crypto/sha256)"
SCALAR_KIND = "port"


def cpu_baseline(w, seconds: float):
    """Oracle (scalar C, 1 thread: the reference's single hash goroutine, mirbft.go:470)
    on a bounded prefix sample of the same workload; plus the strongest CPU numbers:
    OpenSSL libcrypto (SHA-NI) on 1 and CPU_THREADS threads, same sample shape."""
    from oracle import oracle
    oracle.lib()
    n = min(w.n, 4096)
    off, ln = w.off[:n], w.len[:n]
    per = int(ln.sum())
    v, g, done, el = _time_cpu(lambda: oracle.digest_batch(w.arena, off, ln), n, per, seconds / 2)
    line = {"value": None, "unit": "digests/s", "cores": 1, "kind": SCALAR_KIND, "impl": None, "gbps": None,
            "scalar_port": {"value": v, "gbps": g, "source": "oracle/sha256_oracle.c, plain scalar C, 1 thread"},
            "sample": f"first {n} messages of the same workload, repeated for {el:.1f} s "
                      f"({done} digests) per leg"}
    try:
        import platform
        cpu = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")),
                   platform.processor())
        sha_ni = " sha_ni " in open("/proc/cpuinfo").read().replace("\n", " ")
        v1, g1, _, _ = _time_cpu(lambda: oracle.openssl_digest_batch(w.arena, off, ln, 1), n, per, seconds / 2)
        # value: the reference's loop (serial.go:180-198) on ONE core (its single hash
        # goroutine, mirbft.go:470) with the fastest SHA-256 this host has (OpenSSL,
        # SHA-NI): Go 1.15's AVX2 crypto/sha256 would be slower, the scalar port slower still
        line["value"], line["gbps"], line["kind"] = v1, g1, OPENSSL_KIND
        line["impl"] = ("openssl-sha-ni-1-thread (proxy for Go crypto/sha256): the oracle's restatement of "
                        "serial.go:180-198 in C over OpenSSL EVP SHA-256, oracle/sha256_openssl.c")
        m = min(w.n, 4096 * CPU_THREADS)
        offm, lnm = w.off[:m], w.len[:m]
        vt, gt, _, _ = _time_cpu(lambda: oracle.openssl_digest_batch(w.arena, offm, lnm, CPU_THREADS), m,
                                 int(lnm.sum()), seconds / 2)
        line["openssl"] = {"cpu": cpu, "sha_ni": sha_ni,
                           "1_thread": {"value": v1, "gbps": g1},
                           f"{CPU_THREADS}_threads": {"value": vt, "gbps": gt},
                           "source": "oracle/sha256_openssl.c (EVP_Digest*): the fastest CPU SHA-256 on this "
                                     "host (SHA-NI), a strong stand-in for the reference's Go crypto/sha256, "
                                     "which cannot be built here"}
    except (OSError, RuntimeError) as e:   # libcrypto missing: report the port only
        line["openssl"] = {"error": str(e)}
        line["value"], line["gbps"] = v, g
        line["impl"] = "scalar C restatement of serial.go:180-198 over FIPS 180-4, oracle/sha256_oracle.c"
    return line


PMC_FILE = "profiles/r06_pmc.json"          # tools/pmc_valu.sh -> tools/pmc_summary.py, this round's code


def measured_traffic(cfg: str):
    """HBM bytes per step from the committed PMC profile of this round's kernels
    (FETCH_SIZE x the gfx950 calibration + WRITE_SIZE, separate rocprofv3 passes;
    a step's bytes summed over its kernels); (bytes, source) or (None, None)."""
    try:
        with open(os.path.join(ROOT, PMC_FILE)) as f:
            return json.load(f)["configs"][f"{cfg}_auto"]["hbm_bytes"], PMC_FILE
    except (OSError, KeyError, ValueError):
        return None, None


PEAK_CLOCK_GHZ = 2.4


def clock_reading(eng) -> dict:
    """The clock the GPU holds right AFTER a timed region: msha_clock_probe (a
    ~1 ms probe kernel with the hash kernels' VALU mix at 8 waves per SIMD,
    in-kernel s_memtime / s_memrealtime; the hash kernels carry no stamps). A
    diagnostic only: it is not the clock the timed launches ran at (round 5's
    c5 probe read 2.28 GHz after launches that ran nearer 2.4), so no fraction
    is derived from it (tools/lane_stamps.py measures the clock inside the
    launches of a diagnostic build)."""
    try:
        c = eng.clock_probe()
    except Exception as e:  # noqa: BLE001 -- a diagnostic, never fatal to the line
        return {"error": repr(e)[:200]}
    return {"effective_clock_ghz": c["ghz_median"], "min": c["ghz_min"], "max": c["ghz_max"],
            "probe_ms": c["kernel_ms"], "probe_gblocks_per_s": c["gblocks_per_s"],
            "method": "msha_clock_probe right after the timed steps: median over workgroups of "
                      "d(s_memtime) / d(s_memrealtime) x 100 MHz (a separate probe kernel, not the "
                      "timed launches: diagnostic, no fraction is derived from it)"}


def verify_sample(w, d_out, k: int = 512) -> None:
    """Spot-check the timed launches' output against the oracle: k digests at a
    stride that is not a multiple of 64, so every lane position of a wave is hit."""
    from oracle import oracle
    stride = max(1, w.n // k)
    if stride % 64 == 0:
        stride += 1
    sel = np.arange(0, w.n, stride, dtype=np.int64)[:k]
    sel[-1] = w.n - 1
    got = d_out.cpu().numpy()[sel] if hasattr(d_out, "cpu") else d_out[sel]
    exp = oracle.digest_batch(w.arena, w.off[sel], w.len[sel])
    if not np.array_equal(got, exp):
        raise SystemExit(f"bench output mismatch vs oracle ({int((got != exp).any(1).sum())} of {sel.size})")


def launch_ranks(args) -> int:
    """--gpus N > 1 without a torchrun environment: start N rank processes (a
    child torchrun, before this process touches any GPU) and return its exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def host_api_leg(args, world: int, unaliased: bool = False) -> dict:
    """The north-star host path over the job's N GPUs, reported beside the
    headline: ONE process, one libmirsha context over device_mask (1 << N) - 1,
    c5's 2^23 mixed actions (strong scaling: the node's storm split over its
    GPUs by cumulative blocks) from a pinned arena through msha_digest_batch,
    digests straight back into pinned memory (bench.py --mode lib). Run as a
    child process after the ranks have released their GPUs, so a failure there
    costs this object, never the headline line."""
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    gpus = world
    if args.share_device:       # ranks on one GPU: its virtual shards stand in for the GPUs
        env["MSHA_VIRTUAL_SHARDS"] = str(world)
        gpus = 1
    cmd = [sys.executable, os.path.abspath(__file__), "--mode", "lib", "--config", "c5", "--gpus", str(gpus),
           "--steps", "3" if unaliased else "5", "--warmup", "1" if unaliased else "2"]
    if unaliased:
        cmd.append("--unaliased")
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode != 0 or not lines:
            return {"error": f"rc={r.returncode}", "stderr_tail": r.stderr[-400:]}
        d = json.loads(lines[-1])
    except Exception as e:  # noqa: BLE001 -- reported, never fatal to the headline
        return {"error": repr(e)[:400]}
    what = ("c5 2^23 mixed actions, pinned arena -> msha_digest_batch -> pinned digests, one process, "
            "one context over all the job's GPUs (PCIe-inclusive; NOT the headline); ")
    what += ("every action packs its own copy of its payload, in action order: 20+ GB of EpochChange "
             "re-hashes cross PCIe (a caller that does not share payloads)" if unaliased else
             "each distinct EpochChange payload packed once and named by every action that carries it "
             "(what the Go drop-in packs since round 4: epochChangeAliases)")
    return host_api_summary(d, what)


def host_api_summary(d: dict, what: str) -> dict:
    """The host_api object from a --mode lib line: the call's figures and, per GPU,
    its shard's messages, lanes, heads, H2D bytes and times -- and its upload rate
    (h2d_bytes / upload_ms), so a node whose links or NUMA placement contend shows
    it GPU by GPU (upload_gbps_min / _max)."""
    per = []
    for x in d["last_call_shards"]:
        e = {k: x[k] for k in ("device", "messages", "lanes", "head_lanes", "h2d_bytes", "device_ms",
                               "upload_ms", "kernel_ms", "first_launch_ms", "plan_kernel_ms")}
        e["upload_gbps"] = x["h2d_bytes"] / x["upload_ms"] / 1e6 if x["upload_ms"] > 0 else None
        per.append(e)
    rates = [e["upload_gbps"] for e in per if e["upload_gbps"] is not None]
    return {"what": what, "arena_bytes": d["arena_bytes"],
            "value": d["value"], "unit": "digests/s", "n_gpus": d["n_gpus"], "shards": d["shards"],
            "virtual_shards": d["virtual_shards"], "ms_per_call": d["ms_per_step"], "call_ms": d["call_ms"],
            "gbps_hashed": d["gbps_hashed"], "steps": d["steps"], "plan_ms": d["last_call_stats"]["plan_ms"],
            "first_launch_ms_max": max(x["first_launch_ms"] for x in d["last_call_shards"]),
            "upload_gbps_min": min(rates) if rates else None, "upload_gbps_max": max(rates) if rates else None,
            "per_gpu": per}


def kind_of(st0: dict, st1: dict) -> str:
    """The kernel(s) the timed launches ran, from the msha_stats launch counters
    (the chain kernels are counted in launches_coop too: "coop" names only the
    cooperative kernel itself)."""
    d = {k: st1[k] - st0[k] for k in ("launches_lane", "launches_pipe", "launches_coop", "launches_split",
                                      "launches_dod", "launches_chain2", "launches_chain8", "launches_lane_ws")}
    d["launches_coop"] -= d["launches_chain2"] + d["launches_chain8"]
    d["launches_lane"] -= d["launches_lane_ws"]
    names = {"launches_lane": "lane", "launches_lane_ws": "lane_ws", "launches_pipe": "pipe", "launches_coop": "coop",
             "launches_chain2": "chain2", "launches_chain8": "chain8",
             "launches_split": "split", "launches_dod": "digest_of_digests"}
    ran = [v for k, v in names.items() if d[k] > 0]
    return "+".join(ran) if ran else "none"


def kernel_step(eng, w, cfg: str, dev, stream):
    """Upload workload w (kernel-resident) and return (step, d_out): one launch
    over the whole batch on `stream`."""
    import torch
    d_out = torch.empty((w.n, 32), dtype=torch.uint8, device=dev)
    if cfg == "c3dd":
        d_table = torch.from_numpy(np.ascontiguousarray(w.table)).to(dev)
        d_idx = torch.from_numpy(w.idx.view(np.int32)).to(dev)
        d_begin = torch.from_numpy(w.begin.view(np.int64)).to(dev)

        def step():
            eng.digest_of_digests_device(d_table, d_idx, d_begin, d_out, stream)
        return step, d_out
    d_arena = torch.from_numpy(w.arena).to(dev)
    if cfg.startswith("u:"):
        def step():
            eng.digest_uniform_device(d_arena, w.uniform_stride, int(w.len[0]), w.n, d_out, stream)
        return step, d_out
    d_off = torch.from_numpy(w.off.view(np.int64)).to(dev)
    d_len = torch.from_numpy(w.len.view(np.int64)).to(dev)
    if cfg in ("c5_planned", "c5_folded"):
        fold = cfg == "c5_folded"

        def step():
            eng.digest_batch_device_planned(d_arena, d_off, d_len, d_out, stream, fold=fold)
        return step, d_out
    d_order = None
    if not w.uniform_stride:
        # mixed sizes: the packer's size-class order (host, once; part of packing)
        from mirbft_amd.engine import order_by_blocks
        d_order = torch.from_numpy(order_by_blocks(w.len).view(np.int32)).to(dev)

    def step():
        eng.digest_batch_device(d_arena, d_off, d_len, d_out, stream, order=d_order)
    return step, d_out


def time_steps(step, args, dev, stream, barrier=None):
    """W warmup steps + untimed steps until min_warmup_ms, then K timed steps
    bracketed by (barrier +) synchronize. Returns (elapsed_s, kernel_ms_mean,
    warmup_steps_run, warmup_ms)."""
    import torch
    tw = time.perf_counter()
    warm = 0
    for _ in range(args.warmup):
        step()
        warm += 1
    torch.cuda.synchronize(dev)
    while (time.perf_counter() - tw) * 1e3 < args.min_warmup_ms:
        for _ in range(8):
            step()
            warm += 1
        torch.cuda.synchronize(dev)
    warmup_ms = (time.perf_counter() - tw) * 1e3
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps if args.events == "step" else 1)]
    if barrier:
        barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if args.events == "step":
        for e0, e1 in evs:
            e0.record(stream)
            step()
            e1.record(stream)
    else:
        evs[0][0].record(stream)
        for _ in range(args.steps):
            step()
        evs[0][1].record(stream)
    torch.cuda.synchronize(dev)
    # This rank's span ends when its GPU has drained; the closing barrier (and
    # the max over ranks) then gives the job's makespan without charging the
    # control-plane barrier's own latency to the hash path.
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    if args.events == "span":
        kern_ms /= args.steps
    return elapsed, kern_ms, warm, warmup_ms


def algorithmic_bytes(w, cfg: str) -> int:
    """HBM bytes one launch must move: payload read + metadata read + digests written.
    Arena forms: payload + off/len (16 B) + order (4 B, mixed sizes) + 32 B out per
    message; digest-of-digests (c3dd): 32 B per part digest + its 4-B index, 8 B per
    begin entry, 32 B out per Batch."""
    if cfg == "c3dd":
        parts = int(w.idx.size)
        return 32 * parts + 4 * parts + 8 * (w.n + 1) + 32 * w.n
    order = 0 if w.uniform_stride else 4 * w.n
    meta = 0 if cfg.startswith("u:") else 16 * w.n + order
    return w.message_bytes + meta + 32 * w.n


def hashed_blocks(w, cfg: str) -> int:
    """Blocks one launch compresses: every message's, or with alias folding
    (c5_folded) each distinct (off, len) once."""
    if cfg != "c5_folded":
        return w.blocks
    key = np.stack([w.off, w.len], axis=1)
    uniq = np.unique(key, axis=0)
    L = uniq[:, 1]
    return int(((L >> np.uint64(6)) + np.where((L & np.uint64(63)) < 56, 1, 2).astype(np.uint64)).sum())


def roofline(w, kern_ms: float, cfg: str, clock: dict | None = None) -> dict:
    achieved = OPS_PER_BLOCK * hashed_blocks(w, cfg) / (kern_ms * 1e-3) / 1e12
    traffic, src = measured_traffic(cfg)
    ghz = (clock or {}).get("effective_clock_ghz")
    return {"bound": "valu", "achieved": achieved, "peak": PEAK_VALU_TOPS,
            "unit": "Tint32op/s", "frac": achieved / PEAK_VALU_TOPS,
            "effective_clock_ghz_after": ghz,
            "traffic": traffic, "traffic_source": src, "ops_per_block": OPS_PER_BLOCK,
            "note": "peak = full-rate int32 VALU (VOP2/v_bitop3, 2 cycles per wave64 "
                    "instr at 2.4 GHz); SHA-256's mix is ~60% half-rate ops (v_alignbit, "
                    "v_add3) and costs ~3.9-4.1 SIMD cycles per instruction on gfx950 "
                    "(DESIGN.md, profiles/r01_valu_microbench*, r01_pmc.json)",
            "algorithmic_bytes_per_launch": algorithmic_bytes(w, cfg),
            "bare_loop_reference": BARE_LOOP_TOPS,
            "frac_of_bare_loop": achieved / BARE_LOOP_TOPS}


def extra_config(eng, cfg: str, args, dev, stream, w=None) -> dict:
    """One more config timed like the headline (kernel-resident, same warmup and
    K), with its own roofline fraction and a verified sample: puts c3/c4 under
    the driver's clock next to c2 (c3, c4 and c5's three forms in the default
    run; w: a workload already built, shared by the c5 forms)."""
    import torch
    if w is None:
        w = build_workload(cfg, 0, 1)
    step, d_out = kernel_step(eng, w, cfg, dev, stream)
    st0 = eng.stats()
    elapsed, kern_ms, warm, warmup_ms = time_steps(step, args, dev, stream)
    clock = clock_reading(eng)
    eng.device_status()
    kind = kind_of(st0, eng.stats())
    verify_sample(w, d_out)
    rf = roofline(w, kern_ms, cfg, clock)
    out = {"workload": w.name, "value": w.n * args.steps / elapsed, "unit": "digests/s",
           "gbps_hashed": w.message_bytes * args.steps / elapsed / 1e9,
           "ms_per_step": elapsed / args.steps * 1e3, "kernel_ms_mean": kern_ms, "kernel": kind,
           "frac": rf["frac"], "achieved": rf["achieved"], "traffic": rf["traffic"],
           "traffic_source": rf["traffic_source"], "effective_clock_ghz_after": rf["effective_clock_ghz_after"],
           "blocks": w.blocks, "hashed_blocks": hashed_blocks(w, cfg),
           "verified": "512 digests vs oracle (stride not a multiple of 64)",
           "warmup_steps_run": warm}
    if cfg in C5_FORMS:
        out["form"] = C5_FORM_NOTES[cfg]
    del step, d_out
    torch.cuda.empty_cache()
    return out


def extra_c5_ranks(eng, args, dev, stream, rank: int, world: int, dist, form: str = "c5", w=None) -> dict:
    """BASELINE config c5 as quoted -- the node's 2^23-action storm split over the
    job's GPUs (strong scaling: each rank hashes its 2^23 / N slice, the same
    generator stream bench.py's one-GPU c5 leg uses) -- kernel-resident, timed
    like the headline: barrier + synchronize around K launches per rank, the max
    over ranks, in one of the C5_FORMS. Every rank verifies 512 of its digests
    against the oracle."""
    import torch
    if w is None:
        w = build_workload("c5", rank, world)
    step, d_out = kernel_step(eng, w, form, dev, stream)
    st0 = eng.stats()
    elapsed, kern_ms, warm, _ = time_steps(step, args, dev, stream, barrier=dist.barrier)
    clock = clock_reading(eng)
    dist.barrier()
    eng.device_status()
    kind = kind_of(st0, eng.stats())
    verify_sample(w, d_out)
    del step, d_out
    torch.cuda.empty_cache()
    lmax = int(w.len.max()) if w.n else 0
    out = c5_rank_summary(dist, world, form, n=w.n, nbytes=w.message_bytes, blocks=w.blocks,
                          hashed=hashed_blocks(w, form),
                          max_blocks=(lmax >> 6) + (1 if (lmax & 63) < 56 else 2) if w.n else 0,
                          elapsed=elapsed, kern_ms=kern_ms, clock_ghz=clock.get("effective_clock_ghz"),
                          steps=args.steps)
    out.update({"workload": f"c5: {1 << 23} mixed actions (70/25/5) over {world} GPUs, {w.n} per GPU",
                "kernel": kind, "warmup_steps_run": warm,
                "verified": "512 digests per rank vs oracle (stride not a multiple of 64)"})
    return out


# The head's cost of one chain block, shader cycles, per planned form: a rank's
# longest payload on its head takes ~blocks x this / clock. Folded, the early head
# runs on the eight-lane kernel (k_digest_chain8: 1,427 blocks in 1.78 ms beside the
# lane kernel at ~2.36 GHz, profiles/r05_fold/early_head_race/, r05_chain8/ring/);
# unfolded, on the cooperative kernel (k_digest_coop: 2.51 ms at ~2.35 GHz,
# profiles/r05_planned_n8/).
HEAD_CYCLES_PER_BLOCK = {"c5_planned": 4150, "c5_folded": 2950}


def c5_rank_summary(dist, world: int, form: str, *, n, nbytes, blocks, hashed, max_blocks, elapsed, kern_ms,
                    clock_ghz, steps) -> dict:
    """The N-rank c5 figures from each rank's own (every rank calls it): the job's
    digests/s over the slowest rank's time, the roofline fraction of N GPUs' peak,
    and, rank by rank, its kernel time, its longest payload and the estimated share
    of its time that payload's serial chain takes on its head (the floor
    of strong scaling: DESIGN.md (e)) -- so the driver's 8-GPU node shows which
    rank and what bounds it."""
    import torch
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_max, kern_max = (float(x) for x in t.tolist())
    tot = torch.tensor([n, nbytes, blocks, hashed], dtype=torch.float64)
    dist.all_reduce(tot)
    tn, tbytes, tblocks, thashed = (float(x) for x in tot.tolist())
    mine = torch.tensor([kern_ms, float(max_blocks), float(clock_ghz or 0.0), float(n)], dtype=torch.float64)
    every = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(every, mine)
    per_kern = [float(e[0]) for e in every]
    per_max = [int(e[1]) for e in every]
    per_clock = [float(e[2]) or PEAK_CLOCK_GHZ for e in every]
    achieved = OPS_PER_BLOCK * thashed / (kern_max * 1e-3) / 1e12      # all GPUs, slowest rank's launch
    out = {"form": C5_FORM_NOTES.get(form, form), "n_gpus": world, "scaling": "strong",
           "value": tn * steps / elapsed_max, "unit": "digests/s",
           "gbps_hashed": tbytes * steps / elapsed_max / 1e9, "ms_per_step": elapsed_max / steps * 1e3,
           "kernel_ms_mean_max_over_ranks": kern_max,
           "frac": achieved / (PEAK_VALU_TOPS * world), "achieved": achieved, "peak": PEAK_VALU_TOPS * world,
           "blocks": int(tblocks), "hashed_blocks": int(thashed),
           "effective_clock_ghz_rank0": clock_ghz,
           "kernel_ms_per_rank": per_kern, "messages_per_rank": [int(e[3]) for e in every],
           "max_blocks_per_rank": per_max}
    if form in ("c5_planned", "c5_folded"):
        cyc = HEAD_CYCLES_PER_BLOCK[form]
        est = [b * cyc / (c * 1e6) for b, c in zip(per_max, per_clock)]
        out["head_chain_ms_est_per_rank"] = est
        out["head_share_est_per_rank"] = [e / k if k > 0 else None for e, k in zip(est, per_kern)]
        out["head_chain_note"] = ("a rank's longest payload on its head: max_blocks x %d cycles (%s, measured in "
                                  "situ) / the rank's measured clock; share = that / the rank's kernel_ms (near 1: "
                                  "the chain bounds the rank)"
                                  % (cyc, "k_digest_chain8" if form == "c5_folded" else "k_digest_coop"))
    return out


def run_lib(args):
    """North-star host path in one process: one libmirsha context over N GPUs
    (device_mask, or MSHA_VIRTUAL_SHARDS shards of one GPU), batch packed in a
    pinned arena as the cgo adapter does, msha_digest_batch per step."""
    import torch  # noqa: F401  (one HIP runtime: torch's, loaded before libmirsha)
    from mirbft_amd import Engine, _lib
    lib_build = _lib.require_tree_build("bench.py --mode lib")
    n_gpus = args.gpus
    eng = Engine((1 << n_gpus) - 1)
    eng.set_kernel_policy(args.policy)
    shards = len(eng.shard_stats())
    w = build_workload(args.config, 0, 1) if args.config == "c5" else None
    if w is None:   # per-GPU batch fixed (weak scaling): N x the one-GPU batch, one call
        from mirbft_amd import workloads as W
        base = {"c2": 1 << 20, "c3": 200_000, "c4": 65536}[args.config]
        w = {"c2": W.c2_requests, "c3": W.c3_batches, "c4": W.c4_large}[args.config](n=base * shards)
    arena, off, ln = w.arena, w.off, w.len
    out = np.empty((w.n, 32), dtype=np.uint8)
    if args.unaliased:
        # every action its own copy of its payload, packed in action order, pinned
        from mirbft_amd import workloads as W
        new_off, total = W.unaliased_layout(w)
        pa = eng.pinned_empty(total + 64)
        pa[total:] = 0
        W.fill_unaliased(w, new_off, pa)
        w = W.Workload(w.name + ", unaliased (each action its own payload copy, action order)", pa, new_off, w.len)
        arena, off, ln = pa, None, None
    if not args.pageable:
        # what the cgo adapter does: payloads, off/len and the digests all in
        # msha_pinned_alloc memory, so every transfer is a DMA of the caller's bytes
        def pinned(a):
            p = eng.pinned_empty(a.nbytes).view(a.dtype).reshape(a.shape)
            p[...] = a
            return p
        arena = w.arena if args.unaliased else pinned(w.arena)
        off, ln = pinned(w.off), pinned(w.len)
        out = eng.pinned_empty(w.n * 32).reshape(w.n, 32)
    for _ in range(max(1, args.warmup)):
        eng.digest_batch(arena, off, ln, out=out)
    calls = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        t1 = time.perf_counter()
        eng.digest_batch(arena, off, ln, out=out)
        calls.append((time.perf_counter() - t1) * 1e3)
    el = time.perf_counter() - t0
    st = eng.stats()
    sh = eng.shard_stats()
    verify_sample(w, out)
    print(json.dumps({
        "metric": "end-to-end host API msha_digest_batch (pack + H2D + kernel + D2H), NOT the headline",
        "mode": "lib", "arena": "pageable numpy" if args.pageable else "pinned (msha_pinned_alloc), off/len pinned",
        "unaliased": bool(args.unaliased), "arena_bytes": int(w.arena.size),
        "value": w.n * args.steps / el, "unit": "digests/s", "n_gpus": n_gpus, "shards": shards,
        "virtual_shards": os.environ.get("MSHA_VIRTUAL_SHARDS"),
        "gbps_hashed": w.message_bytes * args.steps / el / 1e9, "steps": args.steps,
        "ms_per_step": el / args.steps * 1e3, "call_ms": [round(c, 2) for c in calls],
        "config": {"workload": w.name, "config": args.config},
        "scaling": "strong" if args.config == "c5" else "weak",
        "last_call_stats": st, "last_call_shards": sh, "library": lib_build}), flush=True)
    eng.close()


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if args.mode == "kernel" and args.gpus > 1 and world_env is None:
        sys.exit(launch_ranks(args))
    if world_env is not None and int(world_env) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world_env}: launch one rank per GPU")
    if args.mode == "lib":
        return run_lib(args)
    import torch
    import torch.distributed as dist

    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # Control plane only (rendezvous, barrier, max-over-ranks): the hash path
        # has no data exchange between GPUs, so no RCCL communicator is created.
        # Gloo prints its connection handshake on stdout; keep stdout to rank 0's
        # one JSON line.
        sys.stdout.flush()
        saved, devnull = os.dup(1), os.open(os.devnull, os.O_WRONLY)
        os.dup2(devnull, 1)
        try:
            dist.init_process_group("gloo")
        finally:
            os.dup2(saved, 1)
            os.close(saved)
            os.close(devnull)
    if args.share_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from mirbft_amd import Engine, _lib
    # the numbers are the product's only on the tree's own build (never an A/B variant's)
    lib_build = _lib.require_tree_build("bench.py")
    eng = Engine(1 << local)
    eng.set_kernel_policy(args.policy)
    w = build_workload(args.config, rank, world)
    # A dedicated stream: the launches and the timing events share it (torch's
    # default stream has handle 0, which the C ABI reads as "context stream").
    stream = torch.cuda.Stream(dev)
    step, d_out = kernel_step(eng, w, args.config, dev, stream)
    st0 = eng.stats()
    elapsed, kern_ms, warm, warmup_ms = time_steps(step, args, dev, stream,
                                                   barrier=dist.barrier if world > 1 else None)
    clock = clock_reading(eng)
    if world > 1:
        dist.barrier()
    eng.device_status()
    kind = kind_of(st0, eng.stats())
    if not (args.config.startswith("u:") and w.uniform_stride != (int(w.len[0]) + 15) // 16 * 16):
        verify_sample(w, d_out)

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        counts = torch.tensor([w.n, w.message_bytes, w.blocks], dtype=torch.float64)
        dist.all_reduce(counts)
        tot_n, tot_bytes, _ = (float(x) for x in counts.tolist())
    else:
        tot_n, tot_bytes = float(w.n), float(w.message_bytes)

    if rank == 0:
        value = tot_n * args.steps / elapsed
        gbps = tot_bytes * args.steps / elapsed / 1e9
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "digests/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_steps_run": warm,
            "warmup_ms": warmup_ms,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.config in C5_FORMS else "weak",  # c5: 8M actions per node
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 seed 0x4D49524246540000), inputs resident in HBM",
            "config": {"workload": w.name, "config": args.config, "messages_per_gpu": w.n,
                       "message_bytes_per_gpu": w.message_bytes, "blocks_per_gpu": w.blocks,
                       "hashed_blocks_per_gpu": hashed_blocks(w, args.config),
                       "max_blocks_per_message": int((int(w.len.max()) >> 6) + (1 if (int(w.len.max()) & 63) < 56
                                                                                  else 2)) if w.n else 0,
                       "parallelism": f"independent shards x{world}"},
            "gbps_hashed": gbps,
            "kernel_ms_mean": kern_ms,
            "kernel": kind,
            "clock_after": clock,
            "library": lib_build,
            "roofline": roofline(w, kern_ms, args.config, clock),
        }
        if world == 1 and args.config == "c2" and not args.no_extra:
            del step, d_out
            torch.cuda.empty_cache()
            line["extra_configs"] = {c: extra_config(eng, c, args, dev, stream) for c in ("c3", "c4")}
            w5 = build_workload("c5", 0, 1)
            for c in C5_FORMS:
                line["extra_configs"][c] = extra_config(eng, c, args, dev, stream, w5)
            del w5
    if world > 1 and args.config == "c2" and not args.no_extra:
        # every rank takes part: c5 is quoted over the node's GPUs (BASELINE config 5)
        del step, d_out
        torch.cuda.empty_cache()
        w5 = build_workload("c5", rank, world)
        c5 = {c: extra_c5_ranks(eng, args, dev, stream, rank, world, dist, c, w5) for c in C5_FORMS}
        del w5
        if rank == 0:
            line["extra_configs"] = c5
    eng.close()
    if world > 1:
        dist.barrier()              # every rank has released its GPU
        dist.destroy_process_group()
    if rank == 0:
        if not args.no_cpu_baseline:
            # on the host cores, after every rank has released its GPU
            line["cpu_baseline"] = cpu_baseline(w, args.cpu_seconds)
        if not args.no_host_api:
            line["host_api"] = host_api_leg(args, world)
            if not args.no_host_api_unaliased:
                line["host_api_unaliased"] = host_api_leg(args, world, unaliased=True)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
