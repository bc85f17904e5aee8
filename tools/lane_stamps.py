#!/usr/bin/env python3
"""Where a hash step's time goes, from inside the kernels.

Runs bench.py's kernel-resident steps (FORMS, default: c2, c5, c5_folded) on a
DIAGNOSTIC build of libmirsha (-DMSHA_LANE_STAMPS, tools/ab_build.sh; loaded with
MSHA_LIB_PATH, never the product library): every wave of the hash kernels stamps
s_memtime / s_memrealtime at its start and end plus the SIMD, CU and XCD it ran on
(kernels.hip "Wave stamps"). After >= WARM_S seconds of back-to-back steps (clocks
settle), ONE step is stamped, and per kernel this prints:

  clock_ghz          sum of the waves' shader cycles / their wall time x 100 MHz
                     (the clock the launch itself ran at; median per wave beside it)
  span_us            first wave start .. last wave end
  first/last start   when the kernel's waves started, relative to the step's first
  waves_per_simd     resident waves per SIMD, averaged over the span (8 = full)
  simds / cus        how many the kernel's waves touched
  timeline           resident waves per SIMD in 20 slices of the span (ramp, tail)

plus the step time of the stamped build (HIP events over STEPS steps) beside it,
since stamping itself costs a little. One JSON line per form on stdout.

    bash tools/lane_stamps.sh        # builds the variant on the box, then runs this
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

KINDS = {1: "lane", 2: "pipe", 3: "chain2", 4: "chain8", 5: "coop"}
REC_WORDS = 8  # kernels.hip WaveStampRec: 64 bytes


def decode(recs: np.ndarray) -> dict:
    t0, r0, t1, r1 = (recs[:, k].astype(np.int64) for k in range(4))
    hw = (recs[:, 4] & 0xFFFFFFFF).astype(np.int64)
    xcc = (recs[:, 4] >> 32).astype(np.int64) & 0xF
    kind = (recs[:, 5] & 0xFFFFFFFF).astype(np.int64)
    block = (recs[:, 5] >> 32).astype(np.int64)
    work = (recs[:, 6] >> 32).astype(np.int64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    cu_key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    return {"t0": t0, "r0": r0, "t1": t1, "r1": r1, "kind": kind, "block": block, "cu": cu_key,
            "simd": cu_key * 4 + simd, "nb": work & 0xFFFF, "lanes": work >> 16}


def simd_busy(simd: np.ndarray, r0: np.ndarray, r1: np.ndarray) -> np.ndarray:
    """Per SIMD: the union of its waves' [r0, r1) intervals (ticks)."""
    order = np.lexsort((r0, simd))
    s, a, b = simd[order], r0[order], r1[order]
    busy = {}
    cur_s, cur_a, cur_b, tot = None, 0, 0, 0
    for k in range(s.size):
        if s[k] != cur_s:
            if cur_s is not None:
                busy[cur_s] = tot + (cur_b - cur_a)
            cur_s, cur_a, cur_b, tot = s[k], a[k], b[k], 0
        elif a[k] > cur_b:
            tot += cur_b - cur_a
            cur_a, cur_b = a[k], b[k]
        else:
            cur_b = max(cur_b, b[k])
    if cur_s is not None:
        busy[cur_s] = tot + (cur_b - cur_a)
    return np.array(list(busy.values()), dtype=np.int64)


def summarize(d: dict, step_r0: int, simds_total: int = 1024) -> dict:
    out = {}
    for k in sorted(set(d["kind"].tolist())):
        m = d["kind"] == k
        r0, r1, t0, t1 = d["r0"][m], d["r1"][m], d["t0"][m], d["t1"][m]
        dr, dt = r1 - r0, t1 - t0
        span = int(r1.max() - r0.min())
        busy = dr >= 100  # waves that ran >= 1 us (idle positions exit at once)
        per_wave = dt[busy] / np.maximum(dr[busy], 1) * 0.1
        e = {"waves": int(m.sum()), "waves_ge_1us": int(busy.sum()),
             "clock_ghz": float(dt[busy].sum() / max(1, dr[busy].sum()) * 0.1) if busy.any() else None,
             "clock_ghz_median_wave": float(np.median(per_wave)) if busy.any() else None,
             "clock_ghz_p10_p90": [float(np.percentile(per_wave, 10)), float(np.percentile(per_wave, 90))]
             if busy.any() else None,
             "span_us": span / 100.0,
             "first_start_us": (int(r0.min()) - step_r0) / 100.0,
             "last_start_us": (int(r0.max()) - step_r0) / 100.0,
             "end_us": (int(r1.max()) - step_r0) / 100.0,
             "simds": int(np.unique(d["simd"][m]).size), "cus": int(np.unique(d["cu"][m]).size),
             "waves_per_simd": float(dr.sum() / max(1, span) / simds_total)}
        # resident waves per SIMD over 20 slices of the kernel's span
        lo, bins = int(r0.min()), 20
        edges = lo + np.arange(bins + 1) * max(1, span) / bins
        tl = []
        for b in range(bins):
            a, z = edges[b], edges[b + 1]
            ov = np.clip(np.minimum(r1, z) - np.maximum(r0, a), 0, None).sum()
            tl.append(round(float(ov / (z - a) / simds_total), 2))
        e["timeline_waves_per_simd"] = tl
        e["wave_us_p10_p50_p90_max"] = [float(np.percentile(dr, q)) / 100.0 for q in (10, 50, 90, 100)]
        if KINDS.get(k) == "lane":
            nb, lanes = d["nb"][m], d["lanes"][m]
            busy_ticks = simd_busy(d["simd"][m], r0, r1)
            clk = e["clock_ghz"] or 2.4
            # SIMD cycles the waves' SIMDs were busy (any wave resident) per wave-block
            # (one wave's pass over one block: ~1,356-1,400 VALU instructions, ~5,500
            # cycles at 4.1 a instruction when the SIMD issues without gaps)
            e["simd_busy_frac"] = float(busy_ticks.sum() / (span * simds_total))
            e["wave_blocks"] = int(nb.sum())
            e["lane_blocks"] = int((nb * lanes).sum())
            e["busy_simd_cycles_per_wave_block"] = float(busy_ticks.sum() / 100.0 * 1e3 * clk / max(1, nb.sum()))
            e["full_lane_share"] = float(lanes.sum() / max(1, 64 * (nb > 0).sum()))
            e["blocks_per_wave_hist"] = {int(b): int(c) for b, c in zip(*np.unique(nb, return_counts=True))
                                         if c >= max(1, m.sum() // 200)}
        out[KINDS.get(k, str(k))] = e
    return out


def main():
    import torch
    from mirbft_amd import Engine, _lib
    from mirbft_amd import workloads as W
    L = _lib.lib()
    if not hasattr(L, "msha_diag_wave_stamps"):
        raise SystemExit("%s has no msha_diag_wave_stamps: build it with -DMSHA_LANE_STAMPS "
                         "(tools/lane_stamps.sh) and load it with MSHA_LIB_PATH" % _lib.LIB_PATH)
    fn = L.msha_diag_wave_stamps
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    per = 1 << 18  # records per kernel kind (c5: 131,072 lane waves)
    buf = torch.zeros(5 * per * REC_WORDS, dtype=torch.int64, device=dev)
    cnt = torch.tensor([0, per], dtype=torch.int32, device=dev)
    assert fn(None, None) == 0
    eng = Engine(1)
    stream = torch.cuda.Stream(dev)
    warm_s = float(os.environ.get("WARM_S", "1.5"))
    steps = int(os.environ.get("STEPS", "20"))
    w5 = None
    for form in os.environ.get("FORMS", "c2 c5 c5_folded").split():
        if form in bench.C5_FORMS:
            w5 = w5 or W.c5_storm(n=int(os.environ.get("C5_N", str(1 << 23))))
            w = w5
        else:
            w = bench.build_workload(form, 0, 1)
        step, d_out = bench.kernel_step(eng, w, form, dev, stream)
        st0 = eng.stats()
        tw = time.perf_counter()
        while time.perf_counter() - tw < warm_s:
            for _ in range(8):
                step()
            torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            step()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        step_ms = e0.elapsed_time(e1) / steps
        # one stamped step, right after the timed ones (clocks still settled)
        buf.zero_()
        torch.cuda.synchronize(dev)
        assert fn(buf.data_ptr(), cnt.data_ptr()) == 0
        step()
        torch.cuda.synchronize(dev)
        assert fn(None, None) == 0
        eng.device_status()
        kind = bench.kind_of(st0, eng.stats())
        bench.verify_sample(w, d_out)
        recs = buf.view(-1, REC_WORDS).cpu().numpy().view(np.uint64)
        recs = recs[recs[:, 0] != 0]
        k = int(recs.shape[0])
        d = decode(recs)
        step_r0 = int(d["r0"].min())
        raw = os.environ.get("RAW_DIR")
        if raw:
            os.makedirs(raw, exist_ok=True)
            np.savez_compressed(os.path.join(raw, f"stamps_{form}.npz"), recs=recs)
        line = {"form": form, "workload": w.name, "library": _lib.build_id()["id"], "kernel": kind,
                "step_ms_stamped_build": step_ms, "records": k,
                "hashed_blocks": bench.hashed_blocks(w, form),
                "step_span_us": (int(d["r1"].max()) - step_r0) / 100.0,
                "kernels": summarize(d, step_r0)}
        lane = line["kernels"].get("lane")
        if lane:
            lane_us = lane["span_us"]
            line["lane_g_blocks_per_s"] = line["hashed_blocks"] / lane_us / 1e3
            line["lane_frac"] = bench.OPS_PER_BLOCK * line["hashed_blocks"] / (lane_us * 1e-6) / 1e12 \
                / bench.PEAK_VALU_TOPS
        print(json.dumps(line), flush=True)
        del step, d_out
        torch.cuda.empty_cache()
    eng.close()


if __name__ == "__main__":
    main()
