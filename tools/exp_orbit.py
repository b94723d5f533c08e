"""Experiment: what camera motion costs the blend.  For orbit steps of 0 .. 0.25 degrees per frame,
time 50 frames (events around the blend on every frame) and report fps and blend us; then the last
orbit camera rendered statically (same view every frame).  Config 2 by default."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsm-renderer_amd"))
import gsm_amd  # noqa: E402
from gsm_amd import scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2_1m_sh3_1080p_f16"
c = scenes.CONFIGS[cfg]
n, W, H, sh, prec = c["count"], c["width"], c["height"], c["sh"], c["precision"]
wn, hn, cam_d = scenes.gen_scene(n, W, H, sh, prec, seed=42)
dev = torch.device("cuda", 0)
world = torch.from_numpy(wn.view(np.uint8).reshape(-1).copy()).to(dev)
harm = torch.from_numpy(hn.view(np.uint8).reshape(-1).copy()).to(dev)
r = gsm_amd.GlobalRenderer(device=0, config=gsm_amd.RendererConfig(max_gaussians=n, max_width=W, max_height=H,
                                                                   precision=prec, gaussian_color_space=0))
color = torch.zeros((H, W, 4), dtype=torch.float16, device=dev)
depth = torch.zeros((H, W), dtype=torch.float16, device=dev)
inp = gsm_amd.GaussianInput(world, harm, n, sh)


def run(cams, label):
    for cm in cams[:5]:
        r.render(color, depth, inp, cm, W, H)
    r.set_profiling(stage_events=False, blend_events=True, blend_event_period=1)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for cm in cams[5:]:
        r.render(color, depth, inp, cm, W, H)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t) / (len(cams) - 5)
    print(f"{label:40s} {1 / el:8.1f} fps  blend {r.stage_times_ms()['blend'] * 1e3:7.1f} us  "
          f"A {r.counters()['total_assignments']}", flush=True)


steps = [float(x) for x in os.environ.get("ORBIT_STEPS", "0,0.01,0.05,0.25,1").split(",")]
for step in steps:
    cams = [gsm_amd.CameraParams.from_dict(scenes.orbit_camera(W, H, step * (i + 1))) for i in range(55)]
    run(cams, f"orbit {step} deg/frame")
last = gsm_amd.CameraParams.from_dict(scenes.orbit_camera(W, H, 0.25 * 55))
run([last] * 55, "static at 13.75 deg")
# alternate two views: each frame's schedule comes from the other view
a, b = (gsm_amd.CameraParams.from_dict(scenes.orbit_camera(W, H, x)) for x in (0.0, 13.75))
run([a, b] * 28, "alternating 0 / 13.75 deg")
