"""Per-unit blend trace on one GPU (gsm_global_set_profiling bit 2): unit start/end times,
entries walked and the wave slot each unit ran on.  Prints occupancy over time and the
time per walked entry, and saves the raw trace to gpurun_out/blend_trace_<config>.npz.

usage: python tools/blend_trace.py [--config cfg2_1m_sh3_1080p_f16]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsm-renderer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2_1m_sh3_1080p_f16")
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--angle", type=float, default=0.0, help="orbit camera angle (scenes.orbit_camera)")
    args = ap.parse_args()
    import torch
    import gsm_amd
    from gsm_amd import scenes
    c = scenes.CONFIGS[args.config]
    n, W, H, sh, prec = c["count"], c["width"], c["height"], c["sh"], c["precision"]
    wnp, hnp, cam = scenes.gen_scene(n, W, H, sh, prec, seed=42)
    dev = torch.device("cuda", 0)
    world = torch.from_numpy(wnp.view(np.uint8).copy()).to(dev)
    harm = torch.from_numpy(hnp.view(np.uint8).copy()).to(dev)
    r = gsm_amd.GlobalRenderer(0, gsm_amd.RendererConfig(max_gaussians=n, max_width=W, max_height=H,
                                                         precision=prec, gaussian_color_space=0))
    color = torch.empty((H, W, 4), dtype=torch.float16, device=dev)
    depth = torch.empty((H, W), dtype=torch.float16, device=dev)
    inp = gsm_amd.GaussianInput(world, harm, n, sh)
    cp = gsm_amd.CameraParams.from_dict(scenes.orbit_camera(W, H, args.angle) if args.angle else cam)
    for _ in range(3):
        r.render(color, depth, inp, cp, W, H)
    r.set_profiling(True, blend_trace=True)
    for _ in range(args.frames):
        r.render(color, depth, inp, cp, W, H)
    torch.cuda.synchronize()
    st = r.stage_times_ms()
    tr = r.copy_buffer(gsm_amd.BufferId.BLEND_TRACE).astype(np.int64)
    hd = r.copy_buffer(gsm_amd.BufferId.HEADERS)
    tr = tr[tr[:, 1] > 0]  # units of this frame (2 per tile at the default pairs-per-lane)
    units = tr.shape[0]
    t0 = tr[:, 0].min()
    start = (tr[:, 0] - t0) * 10.0  # 100 MHz ticks -> ns
    end = (tr[:, 1] - t0) * 10.0
    walked = tr[:, 2] & 0xFFFFFFFF
    count = tr[:, 2] >> 32
    span = end.max()
    dur = end - start
    grid = np.linspace(0, span, 201)
    occ = [int(((start <= x) & (end > x)).sum()) for x in grid[:-1]]
    busy = dur.sum() / (span * max(occ))
    wk = walked > 0
    out = {
        "config": args.config, "angle": args.angle, "units": int(units), "blend_ms_events": st.get("blend"),
        "trace_span_us": span / 1e3, "max_concurrent": int(max(occ)),
        "slot_busy_frac": float(busy),
        "mean_unit_us": float(dur.mean() / 1e3), "max_unit_us": float(dur.max() / 1e3),
        "walked_total": int(walked.sum()), "count_total": int(count.sum()),
        "ns_per_entry_mean": float((dur[wk] / walked[wk]).mean()),
        "occupancy_deciles": [occ[i] for i in range(0, 200, 20)],
        "occupancy_tail": [occ[i] for i in range(180, 200, 2)],
    }
    # per wave slot (XCC_ID << 48 | HW_ID of t[3]): the gaps between a slot's consecutive units
    # (unit end -> next unit's first list load: the order / tile-start / half-count loads)
    t3 = tr[:, 3].astype(np.uint64)
    slot = ((t3 >> np.uint64(48)) << np.uint64(32)) | (t3 & np.uint64(0xFFFFFFFF))
    gaps = []
    for sid in np.unique(slot):
        sel = np.nonzero(slot == sid)[0]
        o = sel[np.argsort(start[sel])]
        if o.size > 1:
            gaps.extend((start[o[1:]] - end[o[:-1]]).tolist())
    gaps = np.array(gaps) if gaps else np.zeros(1)
    out["slots"] = int(np.unique(slot).size)
    out["inter_unit_gap_us_mean"] = float(gaps.mean() / 1e3)
    out["inter_unit_gap_us_p90"] = float(np.percentile(gaps, 90) / 1e3)
    out["gap_frac_of_slot_time"] = float(gaps.sum() / max(1.0, dur.sum() + gaps.sum()))
    print(json.dumps(out))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"blend_trace_{args.config}_{args.angle:g}.npz"), trace=tr)


if __name__ == "__main__":
    main()
