"""Blend time of tile-row slabs (the multi-GPU owner's share of a frame) under create-time blend
variants, on one GPU: one renderer per (variant, slab), stage events, images compared per slab.

usage: python tools/exp_slab.py --config cfg2_1m_sh3_1080p_f16 --waves 0,4,8 --fractions 1,2,4,8
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
    ap.add_argument("--waves", default="0,4,8")
    ap.add_argument("--fractions", default="1,2,4,8")
    ap.add_argument("--frames", type=int, default=20)
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
    color = torch.empty((H, W, 4), dtype=torch.float16, device=dev)
    inp = gsm_amd.GaussianInput(world, harm, n, sh)
    cp = gsm_amd.CameraParams.from_dict(cam)
    tiles_y = (H + 15) // 16
    for frac in [int(x) for x in args.fractions.split(",")]:
        rows = (tiles_y + frac - 1) // frac
        ref = None
        for wv in args.waves.split(","):
            if wv == "0":
                os.environ.pop("GSM_BLEND_WAVES", None)
            else:
                os.environ["GSM_BLEND_WAVES"] = wv
            r = gsm_amd.GlobalRenderer(0, gsm_amd.RendererConfig(max_gaussians=n, max_width=W, max_height=H,
                                                                 precision=prec, gaussian_color_space=0))
            # the middle slab (the densest rows of the synthetic scene)
            r0 = max(0, tiles_y // 2 - rows // 2)
            r.set_tile_rows(r0, min(tiles_y, r0 + rows))
            for _ in range(3):
                r.render(color, None, inp, cp, W, H)
            r.set_profiling(True)
            blend = []
            for _ in range(args.frames):
                r.render(color, None, inp, cp, W, H)
                torch.cuda.synchronize()
                blend.append(r.stage_times_ms()["blend"])
            r.set_profiling(False)
            img = color[r0 * 16:min(H, (r0 + rows) * 16)].view(torch.int16).cpu().numpy().tobytes()
            ref = ref or img
            print(json.dumps({"fraction": frac, "rows": rows, "waves": wv, "blend_us": round(1e3 * float(np.median(blend)), 1),
                              "same_image": img == ref}), flush=True)
            r.close()
    os.environ.pop("GSM_BLEND_WAVES", None)


if __name__ == "__main__":
    main()
