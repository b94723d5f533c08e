"""Per-rank device time of the native multi-GPU frame at world W, from W virtual ranks on one GPU
(gsm_debug_partition_* , include/gsm_debug.h): each rank's partition projection + count, its push
into the slab owners' receive buffers, and each owner's slab render from the received records,
timed with HIP events on one stream (ranks run one after another, so each step sees the whole
GPU -- an upper bound for a rank's own GPU).  No collectives and no xGMI: the push writes local
memory.  Prints JSON: per-step times per rank and max_proj_push + max_render, the device part of
one N-GPU frame.

usage: python tools/exp_virtual_ranks.py [--config cfg3_5m_sh3_4k_f16] [--world 8] [--frames 5]
"""
import argparse
import json
import math
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
    tiles_y = (h + 15) // 16
    per_rows = math.ceil(tiles_y / W)
    rows = [min(i * per_rows, tiles_y) for i in range(W + 1)]
    per_ids = math.ceil(n / W)
    cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
    ranks = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(W)]
    send = [torch.zeros(W, dtype=torch.int32, device=dev) for _ in range(W)]
    recv = [torch.zeros(n * gsm.SPLAT_RECORD_BYTES, dtype=torch.uint8, device=dev) for _ in range(W)]
    rcnt = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in range(W)]
    color = torch.zeros((h, w, 4), dtype=torch.float16, device=dev)
    depth = torch.zeros((h, w), dtype=torch.float16, device=dev)
    for d in range(W):
        ranks[d].set_tile_rows(rows[d], rows[d + 1])
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    proj = np.zeros((a.frames, W))
    push = np.zeros((a.frames, W))
    rend = np.zeros((a.frames, W))
    for f in range(a.frames + 2):
        marks = []
        for rk in range(W):
            first = min(rk * per_ids, n)
            e0, e1 = ev(), ev()
            e0.record()
            ranks[rk].debug_partition_counts(inp, cam, w, h, first, min(per_ids, n - first), rows, send[rk])
            e1.record()
            marks.append(("p", rk, e0, e1))
        counts = torch.stack(send).contiguous()
        for rk in range(W):
            e0, e1 = ev(), ev()
            e0.record()
            ranks[rk].debug_partition_push(W, rk, counts, recv, rcnt[rk])
            e1.record()
            marks.append(("u", rk, e0, e1))
        for d in range(W):
            if rows[d] == rows[d + 1]:
                continue
            e0, e1 = ev(), ev()
            e0.record()
            ranks[d].debug_render_records_device_count(color, depth, recv[d], n, rcnt[d], w, h)
            e1.record()
            marks.append(("r", d, e0, e1))
        torch.cuda.synchronize()
        if f < 2:
            continue
        for kind, rk, e0, e1 in marks:
            t = e0.elapsed_time(e1)
            {"p": proj, "u": push, "r": rend}[kind][f - 2, rk] = t
    cm = counts.cpu().numpy().astype(np.int64)
    out = {"config": a.config, "world": W, "records_per_slab": [int(x) for x in cm.sum(axis=0)],
           "records_total": int(cm.sum()), "project_count_ms": proj.mean(0).round(4).tolist(),
           "push_ms": push.mean(0).round(4).tolist(), "render_ms": rend.mean(0).round(4).tolist(),
           "max_project_push_ms": float((proj + push).mean(0).max()), "max_render_ms": float(rend.mean(0).max()),
           "note": "ranks timed one after another on one GPU (each step has the whole GPU); no collectives, no xGMI"}
    out["device_frame_ms"] = out["max_project_push_ms"] + out["max_render_ms"]
    # stage breakdown of the slowest slab render (stage events on that renderer, 5 more frames)
    d = int(np.argmax(rend.mean(0)))
    ranks[d].set_profiling(stage_events=True)
    for _ in range(5):
        ranks[d].debug_render_records_device_count(color, depth, recv[d], n, rcnt[d], w, h)
    torch.cuda.synchronize()
    out["slowest_slab"] = d
    out["slowest_slab_stages_ms"] = {k: round(v, 4) for k, v in ranks[d].stage_times_ms().items()}
    print(json.dumps(out))
    for r in ranks:
        r.close()


if __name__ == "__main__":
    main()
