"""Per-unit alive-group curves of the Global blend from a GSM_BLEND_ZSTATS=2 library build: for every
unit the first entry after which at most 30, 28, 24, 20, 16, 12, 8, 6, 4, 2, 0 of its 32 groups (16 for
quadrant units) are alive, with the walk and the compaction entry.  Saved to
gpurun_out/blend_curves_<config>_<angle>.npz for tools/blend_pair_model.py.

usage (on a GPU box, lib/libgsm_amd.so = the statistics build):
  python tools/blend_curves.py --config cfg2_1m_sh3_1080p_f16 --angles 0 13.75
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsm-renderer_amd"))
THR = [30, 28, 24, 20, 16, 12, 8, 6, 4, 2, 0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2_1m_sh3_1080p_f16")
    ap.add_argument("--angles", type=float, nargs="+", default=[0.0])
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
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
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
        thr = np.zeros((len(tr), len(THR)), np.int64)
        for i in range(6):
            thr[:, i] = ((tr[:, 0] >> np.uint64(10 * i)) & np.uint64(1023)).astype(np.int64)
        for i in range(6, 11):
            thr[:, i] = ((tr[:, 3] >> np.uint64(10 * (i - 6))) & np.uint64(1023)).astype(np.int64)
        ncomp = ((tr[:, 3] >> np.uint64(50)) & np.uint64(1023)).astype(np.int64)
        path = os.path.join(ROOT, "gpurun_out", f"blend_curves_{args.config}_{ang:g}.npz")
        np.savez_compressed(path, walked=walked, count=count, thr=thr, ncomp=ncomp, thresholds=np.array(THR))
        print(args.config, ang, "units", len(tr), "walked", int(walked.sum()), "->", path, flush=True)
    r.close()


if __name__ == "__main__":
    main()
