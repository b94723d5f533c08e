"""Blend time of one tile-row slab (the per-rank work of an N-GPU frame) on one GPU."""
import os, sys, json
import numpy as np, torch
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, R + "/gsm-renderer_amd")
import gsm_amd
from gsm_amd import scenes, slabs
cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2_1m_sh3_1080p_f16"
c = scenes.CONFIGS[cfg]
n, W, H, sh, prec = c["count"], c["width"], c["height"], c["sh"], c["precision"]
wnp, hnp, cam = scenes.gen_scene(n, W, H, sh, prec, seed=42)
dev = torch.device("cuda", 0)
world = torch.from_numpy(wnp.view(np.uint8).reshape(-1).copy()).to(dev)
harm = torch.from_numpy(hnp.view(np.uint8).reshape(-1).copy()).to(dev)
r = gsm_amd.GlobalRenderer(0, gsm_amd.RendererConfig(max_gaussians=n, max_width=W, max_height=H, precision=prec,
                                                     gaussian_color_space=0))
color = torch.zeros((H, W, 4), dtype=torch.float16, device=dev)
depth = torch.zeros((H, W), dtype=torch.float16, device=dev)
inp = gsm_amd.GaussianInput(world, harm, n, sh)
cp = gsm_amd.CameraParams.from_dict(cam)
tiles_y = (H + 15) // 16
out = {}
for ws in (1, 2, 4, 8):
    worst = 0.0
    for rank in range(ws):
        s = slabs.partition(tiles_y, H, ws, rank)
        r.set_tile_rows(s.row_begin, s.row_end) if ws > 1 else r.set_tile_rows(0, 0)
        for _ in range(4):
            r.render(color, depth, inp, cp, W, H)
        r.set_profiling(stage_events=True)
        for _ in range(10):
            r.render(color, depth, inp, cp, W, H)
        torch.cuda.synchronize()
        st = r.stage_times_ms()
        r.set_profiling(stage_events=False)
        worst = max(worst, st["blend"])
    out[ws] = round(worst * 1000, 1)
print(json.dumps({"config": cfg, "pairs": os.environ.get("GSM_BLEND_PAIRS", "2"), "worst_slab_blend_us": out}))
