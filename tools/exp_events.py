"""Experiment: what do the per-frame blend timing events and the blend schedule's side-stream
join cost?  Renders config 2 frames back to back (wall clock over 200 frames) with: no events,
blend events every frame, and GSM_BLEND_SCHED read per frame (0 = no side stream)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsm-renderer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2_1m_sh3_1080p_f16")
    ap.add_argument("--frames", type=int, default=200)
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
    cp = gsm_amd.CameraParams.from_dict(cam)
    s = torch.cuda.current_stream(dev)
    out = {}
    for name, sched, ev in [("sched_noev", "1", False), ("sched_ev", "1", True), ("nosched_noev", "0", False),
                            ("nosched_ev", "0", True), ("sched_noev2", "1", False)]:
        os.environ["GSM_BLEND_SCHED"] = sched
        r.set_profiling(stage_events=False, blend_events=ev)
        for _ in range(10):
            r.render(color, depth, inp, cp, W, H, stream=s)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.frames):
            r.render(color, depth, inp, cp, W, H, stream=s)
        torch.cuda.synchronize()
        out[name] = round((time.perf_counter() - t) / args.frames * 1e3, 4)
    print(json.dumps({"config": args.config, "ms_per_frame": out}))


if __name__ == "__main__":
    main()
