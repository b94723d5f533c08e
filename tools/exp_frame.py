"""A/B experiments on one GPU: time the frame's stages under several env-var variants,
interleaved in one process (cdna_hip_programming.md 5.4 rule 24).

usage: python tools/exp_frame.py --config cfg2_1m_sh3_1080p_f16 --var GSM_BLEND_WG_WAVES_DYN=16,8,4
"""
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
    ap.add_argument("--var", action="append", default=[])
    ap.add_argument("--rounds", type=int, default=3)
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
    r = gsm_amd.GlobalRenderer(0, gsm_amd.RendererConfig(max_gaussians=n, max_width=W, max_height=H,
                                                         precision=prec, gaussian_color_space=0))
    color = torch.empty((H, W, 4), dtype=torch.float16, device=dev)
    depth = torch.empty((H, W), dtype=torch.float16, device=dev)
    inp = gsm_amd.GaussianInput(world, harm, n, sh)
    cp = gsm_amd.CameraParams.from_dict(cam)
    variants = [("", {})]
    for v in args.var:  # cartesian product of the listed values
        k, vals = v.split("=")
        variants = [(f"{name} {k}={x}".strip(), {**env, k: x}) for name, env in variants
                    for x in vals.split(",")]
    varied = {k for _, env in variants for k in env}
    results = {name: [] for name, _ in variants}
    ref = None
    for rnd in range(args.rounds):
        for name, env in variants:
            for k in list(os.environ):
                if k in varied:
                    del os.environ[k]
            os.environ.update(env)
            for _ in range(3):
                r.render(color, depth, inp, cp, W, H)
            r.set_profiling(True)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(args.frames):
                r.render(color, depth, inp, cp, W, H)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / args.frames * 1e3
            st = r.stage_times_ms()
            r.set_profiling(False)
            img = color.view(torch.int16).cpu().numpy().tobytes()
            if ref is None:
                ref = img
            st["frame_ms"] = ms
            st["same_image"] = img == ref
            results[name].append(st)
    for name, lst in results.items():
        keys = [k for k in lst[0] if k != "same_image"]
        med = {k: float(np.median([x[k] for x in lst])) for k in keys}
        print(json.dumps({"variant": name, "same_image": all(x["same_image"] for x in lst),
                          **{k: round(v, 4) for k, v in med.items()}}))


if __name__ == "__main__":
    main()
