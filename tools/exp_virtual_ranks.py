"""Per-rank device time of the multi-GPU frame at world W, from W virtual ranks on one GPU driven
through the product path (gsm_multigpu_render_phase, include/gsm_multigpu.h): every rank's phase p
is issued before any rank's phase p + 1 on ONE stream, so the ranks run one after another and each
phase sees the whole GPU (an upper bound for a rank's own GPU).  Exchange memory is the product's
(fine-grained, the flag barriers run); the pushes and the gathered pixels go to local memory instead of
crossing xGMI.  HIP events bracket each rank's phase; the renderers' stage events split the slab
render (records in, scan, scatter, sort, gap, blend).

Prints JSON: per-phase times per rank, and device_frame_ms = max phase 0 + max phase 1 + max phase 2
(+ phase 3), the device part of one N-GPU frame without the fabric.  Each timed frame is enqueued while
the GPU spins (--hold-cycles), so no event pair times the host's enqueue of a phase.

usage: python tools/exp_virtual_ranks.py [--config cfg3_5m_sh3_4k_f16] [--world 8] [--frames 5]
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
    ap.add_argument("--config", default="cfg3_5m_sh3_4k_f16")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--stages", type=int, default=1, help="also time the slab render's stages")
    ap.add_argument("--single", type=int, default=0,
                    help="also time the whole frame on one renderer (same scene, same box): one_gpu_frame_ms")
    ap.add_argument("--trace-rank", type=int, default=-1,
                    help="per-unit blend trace of this rank's slab (profiling bit 2) -> gpurun_out/vr_trace_*.npz")
    ap.add_argument("--depth", type=int, default=1, help="gather the r16f depth frame too (product default)")
    ap.add_argument("--hold-cycles", type=float, default=6e6,
                    help="spin the GPU this many cycles (~2.5 ms) before each timed frame while the host enqueues it")
    ap.add_argument("--interval", type=int, default=0,
                    help="also time N frames issued back to back (no events between phases): the group's frame "
                         "interval; run with GSM_MG_PIPELINE=1 in the environment for the pipelined frame")
    a = ap.parse_args()
    import torch
    import gsm_amd as gsm
    from gsm_amd import scenes
    c = scenes.CONFIGS[a.config]
    n, w, h, sh, prec = c["count"], c["width"], c["height"], c["sh"], c["precision"]
    W = a.world
    wnp, hnp, cam_d = scenes.gen_scene(n, w, h, sh, prec, seed=42)
    dev = torch.device("cuda", 0)
    wt = torch.from_numpy(wnp.view(np.uint8).reshape(-1).copy()).to(dev)
    ht = torch.from_numpy(hnp.view(np.uint8).reshape(-1).copy()).to(dev)
    del wnp, hnp
    inp = gsm.GaussianInput(wt, ht, n, sh)
    cam = gsm.CameraParams.from_dict(cam_d)
    cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
    rends = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(W)]
    pre = [gsm.MultiGpuRenderer.prepare(r, k, W) for k, r in enumerate(rends)]
    handles = [hd for _, hd in pre]
    mgs = [m.connect_handles(handles) for m, _ in pre]
    frame_ptr = mgs[0].frame()[0]
    stream = torch.cuda.current_stream(dev)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    ph = np.zeros((a.frames, 4, W))

    def frame(record):
        # (r06) the GPU waits behind a short spin while the host enqueues the frame's 4 x W phases: each
        # event pair then brackets device work only.  Before, rank 0's phase 0 began on an idle GPU, so
        # its pair also timed the host's enqueue of that phase (~35 us: phase 0 0.085 ms for rank 0
        # against 0.049-0.050 for the others, profiles/r06_virtual_ranks_kernel_trace.txt)
        if record:
            torch.cuda._sleep(int(a.hold_cycles))
        marks = []
        for p in range(4):
            for k, m in enumerate(mgs):
                e0, e1 = ev(), ev()
                e0.record(stream)
                m.render_phases([p], None, None, inp, cam, w, h, gather=True, gather_depth=bool(a.depth), stream=stream,
                                gather_target=frame_ptr if k == 0 else None)
                e1.record(stream)
                marks.append((p, k, e0, e1))
        return marks

    piped = os.environ.get("GSM_MG_PIPELINE") == "1"
    if piped:  # phases 0-1 run on the ranks' own streams: per-phase events on the caller's stream see none
        a.frames, a.stages, a.trace_rank = 0, 0, -1
    for f in range(a.frames + 2 if a.frames else 0):
        marks = frame(True)
        torch.cuda.synchronize()
        if f >= 2:
            for p, k, e0, e1 in marks:
                ph[f - 2, p, k] = e0.elapsed_time(e1)
    stages = None
    if a.stages:
        for r in rends:
            r.set_profiling(stage_events=True)
        for _ in range(3):
            frame(False)
        torch.cuda.synchronize()
        names = ["records_in", "scan", "scatter", "sort", "gap", "blend"]
        stages = []
        for r in rends:
            try:
                t = r.stage_times_ms()
                stages.append({nm: round(float(t[k]), 4) for nm, k in zip(names, ["project", "scan", "scatter", "sort", "headers", "blend"])})
            except gsm.RendererError:
                stages.append(None)  # a rank without rows renders nothing
    trace = None
    if a.trace_rank >= 0:
        r = rends[a.trace_rank]
        r.set_profiling(stage_events=False, blend_trace=True)
        for _ in range(2):
            frame(False)
        torch.cuda.synchronize()
        tr = r.copy_buffer(gsm.BufferId.BLEND_TRACE).astype(np.int64)
        tr = tr[tr[:, 1] > 0]
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        np.savez(os.path.join(ROOT, "gpurun_out", f"vr_trace_{a.config}_w{W}_r{a.trace_rank}.npz"), trace=tr)
        t0 = tr[:, 0].min()
        st, en = (tr[:, 0] - t0) * 0.01, (tr[:, 1] - t0) * 0.01  # 100 MHz ticks -> us
        dur, walk = en - st, tr[:, 2] & 0xFFFFFFFF
        span = float(en.max())
        grid = np.linspace(0, span, 11)[:-1] + span / 20
        trace = {"units": int(tr.shape[0]), "span_us": round(span, 1), "max_unit_us": round(float(dur.max()), 1),
                 "mean_unit_us": round(float(dur.mean()), 1), "sum_unit_us": round(float(dur.sum()), 1),
                 "max_walk": int(walk.max()), "mean_walk": round(float(walk.mean()), 1),
                 "occupancy_deciles": [int(((st <= x) & (en > x)).sum()) for x in grid],
                 "first_start_spread_us": round(float(np.sort(st)[min(len(st) - 1, 3000)]), 1)}
    interval = None
    if a.interval:
        # every phase of every rank of N frames, one caller stream, rank 0 gathering into caller tensors
        # (pipelined ranks refuse the library frames as targets); one event pair around all N frames
        cbuf = torch.empty((h, w, 4), dtype=torch.float16, device=dev)
        dbuf = torch.empty((h, w), dtype=torch.float16, device=dev)
        cams = [gsm.CameraParams.from_dict(scenes.orbit_camera(w, h, 0.25 * i)) for i in range(a.interval + 3)]

        def issue(cm):
            for p in range(4):
                for k, m in enumerate(mgs):
                    m.render_phases([p], cbuf if k == 0 else None, dbuf if k == 0 else None, inp, cm, w, h,
                                    gather=True, gather_depth=bool(a.depth), stream=stream)
        for cm in cams[:3]:
            issue(cm)
        torch.cuda.synchronize()
        e0, e1 = ev(), ev()
        e0.record(stream)
        for cm in cams[3:]:
            issue(cm)
        e1.record(stream)
        torch.cuda.synchronize()
        g = e0.elapsed_time(e1) / a.interval
        interval = {"frames": a.interval, "pipelined": os.environ.get("GSM_MG_PIPELINE") == "1",
                    "group_interval_ms": round(g, 4), "per_rank_interval_ms": round(g / W, 4),
                    "note": "W virtual ranks share one GPU: the group's frame interval / W models one rank's "
                            "interval on its own GPU (moving camera, 0.25 deg per frame)"}
    one_gpu = None
    if a.single:  # the same frame on one renderer with the whole frame's rows (bench.py's 1-GPU path)
        one = gsm.GlobalRenderer(device=0, config=cfg)
        color = torch.empty((h, w, 4), dtype=torch.float16, device=dev)
        depth = torch.empty((h, w), dtype=torch.float16, device=dev)
        for _ in range(3):
            one.render(color, depth, inp, cam, w, h, stream=stream)
        torch.cuda.synchronize()
        e0, e1 = ev(), ev()
        e0.record(stream)
        reps = max(a.frames, 5) * 4
        for _ in range(reps):
            one.render(color, depth, inp, cam, w, h, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        one_gpu = e0.elapsed_time(e1) / reps
        one.close()
    med = np.median(ph, axis=0) if ph.shape[0] else np.zeros((4, W))  # [phase][rank]
    # xGMI model (not a measurement: the virtual ranks' pushes and pixels stay in one GPU's HBM).
    # counts[r][s] = records rank r sends to slab s; every cross-rank record is 48 B (SplatRecord)
    # over the (r, s) link; rank 0 receives every other band's pixels (rgba16f + r16f = 10 B) over
    # that rank's link.  MI355X: 7 xGMI links per GPU, ~153 GB/s each, point to point,
    # all links concurrently; the stores stream while the producing kernel runs, so a phase takes
    # at least max(its device time, its busiest link's bytes / 153 GB/s).
    link_gbs = 153.0
    cm = mgs[0].counts().astype(np.int64)
    rec_link = cm * 48
    np.fill_diagonal(rec_link, 0)
    tiles_y = (h + 15) // 16
    per_rows = (tiles_y + W - 1) // W
    band_px = [max(0, min(h, min(tiles_y, (r + 1) * per_rows) * 16) - min(h, min(tiles_y, r * per_rows) * 16)) * w
               for r in range(W)]
    pix_link = [band_px[r] * 10 if r else 0 for r in range(W)]
    t_push = float(rec_link.max()) / (link_gbs * 1e9) * 1e3
    t_pix = float(max(pix_link)) / (link_gbs * 1e9) * 1e3
    mp = [float(med[p].max()) for p in range(4)]
    model_frame = mp[0] + max(mp[1], t_push) + max(mp[2], t_pix) + mp[3]
    xgmi = {"link_gb_per_s": link_gbs, "records_out_bytes_per_rank": [int(x) for x in rec_link.sum(axis=1)],
            "busiest_link_records_bytes": int(rec_link.max()), "rank0_pixel_in_bytes": int(sum(pix_link)),
            "busiest_link_pixel_bytes": int(max(pix_link)), "push_link_ms": round(t_push, 4),
            "pixel_link_ms": round(t_pix, 4), "modelled_frame_ms": round(model_frame, 4),
            "note": "MODEL, not measured: each phase >= its busiest link's bytes at 153 GB/s (7 concurrent "
                    "point-to-point links per GPU); device phases measured on one GPU"}
    out = {"config": a.config, "world": W, "frames": a.frames, "gather_depth": bool(a.depth), "timeouts": [m.status() for m in mgs],
           "counts": mgs[0].counts().tolist(),
           "phase_ms": {f"phase{p}": [round(float(x), 4) for x in med[p]] for p in range(4)},
           "max_phase_ms": [round(float(med[p].max()), 4) for p in range(4)],
           "device_frame_ms": round(float(sum(med[p].max() for p in range(4))), 4),
           "slab_stages_ms": stages, "blend_trace": trace, "interval": interval,
           "xgmi_model": xgmi,
           "one_gpu_frame_ms": round(one_gpu, 4) if one_gpu else None,
           "device_speedup": round(one_gpu / float(sum(med[p].max() for p in range(4))), 3) if one_gpu and not piped else None,
           "note": "virtual ranks on one GPU, product kernels, one stream; no xGMI (pushes and pixels stay local)"}
    print(json.dumps(out))
    for m in mgs:
        m.close()
    for r in rends:
        r.close()


if __name__ == "__main__":
    main()
