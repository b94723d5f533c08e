"""Experiment: does capturing a whole frame (gsm_global_render) into a hipGraph shorten it?
Captures with torch.cuda.CUDAGraph (the renderer enqueues on the capture stream, its side
stream joins through events) and times graph replays against direct renders."""
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
    ap.add_argument("--frames", type=int, default=50)
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
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        for _ in range(5):
            r.render(color, depth, inp, cp, W, H, stream=s)
        torch.cuda.synchronize()
        ref = color.clone()
        t = time.perf_counter()
        for _ in range(args.frames):
            r.render(color, depth, inp, cp, W, H, stream=s)
        torch.cuda.synchronize()
        direct = (time.perf_counter() - t) / args.frames * 1e3
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        r.render(color, depth, inp, cp, W, H, stream=s)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.frames):
        g.replay()
    torch.cuda.synchronize()
    graphed = (time.perf_counter() - t) / args.frames * 1e3
    print(json.dumps({"config": args.config, "direct_ms": direct, "graph_ms": graphed,
                      "same_image": bool(torch.equal(color.view(torch.int16), ref.view(torch.int16)))}))


if __name__ == "__main__":
    main()
