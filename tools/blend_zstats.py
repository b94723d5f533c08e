"""(r06: the switch lives in tools/exp/blend_zstats.patch -- `git apply` it before that build.)  Walk statistics of the Global blend from a GSM_BLEND_ZSTATS=1 library build (the per-unit trace's
t[3] = live pixels summed over entries << 32 | entries on which no live pixel has a nonzero alpha;
t[0] >> 48 = the entry at which the unit compacted).  Prints, per camera angle, the walked entries,
the all-zero entries and the live-pixel fraction of the walk's pixel slots.

usage (on a GPU box, lib/libgsm_amd.so = the statistics build):
  python tools/blend_zstats.py --config cfg2_1m_sh3_1080p_f16 --angles 0 13.75
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
    ap.add_argument("--angles", type=float, nargs="+", default=[0.0, 13.75])
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
    for ang in args.angles:
        cp = gsm_amd.CameraParams.from_dict(scenes.orbit_camera(W, H, ang) if ang else cam)
        r.set_profiling(False)
        for _ in range(3):
            r.render(color, depth, inp, cp, W, H)
        r.set_profiling(True, blend_trace=True)
        r.render(color, depth, inp, cp, W, H)
        torch.cuda.synchronize()
        tr = r.copy_buffer(gsm_amd.BufferId.BLEND_TRACE).astype(np.uint64)
        tr = tr[tr[:, 1] > 0]
        walked = (tr[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
        count = (tr[:, 2] >> np.uint64(32)).astype(np.int64)
        zero = (tr[:, 3] & np.uint64(0xFFFFFFFF)).astype(np.int64)
        alive_px = (tr[:, 3] >> np.uint64(32)).astype(np.int64)
        ncomp = (tr[:, 0] >> np.uint64(48)).astype(np.int64)
        comp = ncomp > 0
        # pixel slots: 256 per entry before compaction (4 px x 64 lanes), 128 after
        pre = np.where(comp, np.minimum(ncomp, walked), walked)
        post = walked - pre
        slots = 256 * pre + 128 * post
        out = {"config": args.config, "angle": ang, "units": int(tr.shape[0]),
               "walked_entries": int(walked.sum()), "list_entries": int(count.sum()),
               "zero_entries": int(zero.sum()), "zero_frac": float(zero.sum() / max(1, walked.sum())),
               "compacted_units": int(comp.sum()), "entries_after_compaction": int(post.sum()),
               "live_pixel_frac_of_slots": float(alive_px.sum() / max(1, slots.sum())),
               "live_pixel_entries": int(alive_px.sum())}
        print(json.dumps(out))
    r.close()


if __name__ == "__main__":
    main()
