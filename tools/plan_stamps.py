#!/usr/bin/env python3
"""Where the folded planner's time goes, from inside its kernels.

Runs bench.py's kernel-resident c5_folded step on a DIAGNOSTIC build of libmirsha
(-DMSHA_PLAN_STAMPS, tools/ab_build.sh; loaded with MSHA_LIB_PATH, never the
product library): thread 0 of every workgroup of k_fold_insert, k_fold_scatter,
k_fold_scan, k_fold_fill and k_fold_longs_gate stamps s_memrealtime (100 MHz) at
its phase boundaries (plan.hip "Planner stamps"). After WARM_S seconds of steps,
ONE step is stamped; per kernel this prints its span from the step's first stamp,
and per phase the workgroups' durations (p10 / p50 / p90 / max, µs) and their sum
over workgroups divided by the span (how many workgroups spent the span there).

k_fold_insert's phases: 0 start, 1 off/len loaded, 2 in-tile prefix max (and the
tile's own post), 3 first pass (fresh so far / candidates listed) and wave 0's
look-back, 4 second pass (the tiles before applied, lanes counted), 5 claims done,
6 key16/apairs written, 7 flushed (bucket counters). Words 8/9: candidates, keys.

    bash tools/plan_stamps.sh     # builds the variant on the box, then runs this
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

KINDS = {0: ("insert", 8), 1: ("scatter", 4), 2: ("scan", 2), 3: ("fill", 2), 4: ("gate", 2)}
PER = 1 << 12  # records per kind (c5: 2,048 insert / scatter tiles)


def phases(recs: np.ndarray, nph: int, step0: int) -> dict:
    t = recs[:, :nph].astype(np.int64)
    ok = (t[:, 0] != 0) & (t[:, nph - 1] != 0)
    t = t[ok]
    if not t.size:
        return {"workgroups": 0}
    span = int(t[:, nph - 1].max() - t[:, 0].min())
    out = {"workgroups": int(ok.sum()), "first_start_us": (int(t[:, 0].min()) - step0) / 100.0,
           "last_start_us": (int(t[:, 0].max()) - step0) / 100.0,
           "end_us": (int(t[:, nph - 1].max()) - step0) / 100.0, "span_us": span / 100.0,
           "wg_us_p50": float(np.median(t[:, nph - 1] - t[:, 0])) / 100.0}
    ph = {}
    for k in range(1, nph):
        d = (t[:, k] - t[:, k - 1]) / 100.0
        ph[f"{k - 1}->{k}"] = {"p10": float(np.percentile(d, 10)), "p50": float(np.median(d)),
                               "p90": float(np.percentile(d, 90)), "max": float(d.max()),
                               "wgs_in_phase": float(d.sum() / max(span / 100.0, 1e-9))}
    out["phases"] = ph
    # resident workgroups over 10 slices of the span
    lo, hi = t[:, 0], t[:, nph - 1]
    edges = t[:, 0].min() + np.arange(11) * max(1, span) / 10
    out["resident_wgs_timeline"] = [round(float(np.clip(np.minimum(hi, edges[b + 1]) - np.maximum(lo, edges[b]),
                                                        0, None).sum() / (edges[b + 1] - edges[b])), 1)
                                    for b in range(10)]
    return out


def main():
    import torch
    from mirbft_amd import Engine, _lib
    from mirbft_amd import workloads as W
    L = _lib.lib()
    if not hasattr(L, "msha_diag_plan_stamps"):
        raise SystemExit("%s has no msha_diag_plan_stamps: build it with -DMSHA_PLAN_STAMPS "
                         "(tools/plan_stamps.sh) and load it with MSHA_LIB_PATH" % _lib.LIB_PATH)
    fn = L.msha_diag_plan_stamps
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_uint32], ctypes.c_int
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    buf = torch.zeros(6 * PER * 16, dtype=torch.int64, device=dev)
    assert fn(None, 0) == 0
    eng = Engine(1)
    stream = torch.cuda.Stream(dev)
    warm_s = float(os.environ.get("WARM_S", "1.5"))
    steps = int(os.environ.get("STEPS", "20"))
    w = W.c5_storm(n=int(os.environ.get("C5_N", str(1 << 23))))
    for form in os.environ.get("FORMS", "c5_folded").split():
        step, d_out = bench.kernel_step(eng, w, form, dev, stream)
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
        buf.zero_()
        torch.cuda.synchronize(dev)
        assert fn(buf.data_ptr(), PER) == 0
        step()
        torch.cuda.synchronize(dev)
        assert fn(None, 0) == 0
        eng.device_status()
        bench.verify_sample(w, d_out)
        recs = buf.view(6, PER, 16).cpu().numpy().view(np.uint64)
        starts = [int(recs[k][recs[k][:, 0] != 0][:, 0].min()) for k in KINDS if (recs[k][:, 0] != 0).any()]
        step0 = min(starts)
        raw = os.environ.get("RAW_DIR")
        if raw:
            os.makedirs(raw, exist_ok=True)
            np.savez_compressed(os.path.join(raw, f"plan_stamps_{form}.npz"), recs=recs)
        line = {"form": form, "workload": w.name, "library": _lib.build_id()["id"],
                "env": {k: v for k, v in os.environ.items() if k.startswith("MSHA_") and k != "MSHA_LIB_PATH"},
                "step_ms_stamped_build": step_ms, "kernels": {}}
        for k, (name, nph) in KINDS.items():
            line["kernels"][name] = phases(recs[k], nph, step0)
        ins = recs[0][(recs[0][:, 0] != 0)]
        if ins.size:
            line["insert_candidates_p50_max"] = [float(np.median(ins[:, 8])), int(ins[:, 8].max())]
            line["insert_keys_p50_max"] = [float(np.median(ins[:, 9])), int(ins[:, 9].max())]
        print(json.dumps(line), flush=True)
        del step, d_out
        torch.cuda.empty_cache()
    eng.close()


if __name__ == "__main__":
    main()
