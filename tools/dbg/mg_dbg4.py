"""Debug: the (8, fp32) virtual-rank frame repeated; gathered vs own-target bands."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "gsm-renderer_amd")]
import torch
import gsm_amd as gsm
import oracle as O
from gsm_amd import scenes
O.build()
refs = {}
for it in range(4):
    for world, n, w, h, prec in [(8, 50_000, 640, 360, 0), (8, 50_000, 640, 360, 1)]:
        sh = 16 if prec else 4
        wn, hn, cam = scenes.gen_scene(n, w, h, sh, prec, seed=78)
        if (prec) not in refs:
            refs[prec] = O.render(wn, hn, sh, cam, w, h, max_gaussians=n)["color"]
        ref = refs[prec]
        wt = torch.from_numpy(wn.view(np.uint8).reshape(-1).copy()).cuda()
        ht = torch.from_numpy(hn.view(np.uint8).reshape(-1).copy()).cuda()
        inp = gsm.GaussianInput(wt, ht, n, sh)
        cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
        rends = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(world)]
        pre = [gsm.MultiGpuRenderer.prepare(r, k, world) for k, r in enumerate(rends)]
        mgs = [m.connect_handles([hd for _, hd in pre]) for m, _ in pre]
        cp = gsm.CameraParams.from_dict(cam)
        for ph in range(4):
            for k, m in enumerate(mgs):
                m.render_phases([ph], None, None, inp, cp, w, h, gather=True)
        torch.cuda.synchronize()
        got = mgs[0].copy_frame(w, h)
        rows_g = np.nonzero(np.any(got != ref, axis=(1, 2)))[0]
        col = torch.full((h, w, 4), float("nan"), dtype=torch.float16, device="cuda")
        for ph in range(4):
            for k, m in enumerate(mgs):
                m.render_phases([ph], col, None, inp, cp, w, h, gather=False)
        torch.cuda.synchronize()
        own = col.view(torch.int16).cpu().numpy().view(np.uint16)
        rows_o = np.nonzero(np.any(own != ref, axis=(1, 2)))[0]
        cnt = [r.counters() for r in rends]
        print(it, world, prec, "gather bad rows", len(rows_g), rows_g[:3].tolist(), "own bad rows", len(rows_o),
              rows_o[:3].tolist(), "assign", [c["total_assignments"] for c in cnt], flush=True)
        for m in mgs:
            m.close()
        for r in rends:
            r.close()
        del wt, ht
