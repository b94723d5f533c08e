"""Debug: poisoned exchange memory; which received records of a slab were never written."""
import os, sys
os.environ["GSM_MG_POISON"] = "1"
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "gsm-renderer_amd")]
import torch
import gsm_amd as gsm
from gsm_amd import scenes
for world, n, w, h, prec in [(8, 50_000, 640, 360, 0), (8, 50_000, 640, 360, 1), (3, 60_000, 1280, 720, 1)]:
    sh = 16 if prec else 4
    wn, hn, cam = scenes.gen_scene(n, w, h, sh, prec, seed=78)
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
    cm = mgs[0].counts().astype(np.int64)
    for k, m in enumerate(mgs):
        nrec = int(cm[:, k].sum())
        ex = m.copy_exchange(4096 + 48 * (nrec + 8))
        recs = ex[4096:].reshape(-1, 48)
        poisoned = np.nonzero(np.all(recs[:nrec] == 0xAB, axis=1))[0]
        cmk = m.copy_exchange(4096)[1024:3072].view(np.uint32).reshape(2, 16, 16)
        print(world, prec, "rank", k, "recv", nrec, "unwritten", len(poisoned), poisoned[:10].tolist(),
              "tail poisoned", bool(np.all(recs[nrec:nrec + 8] == 0xAB)), flush=True)
    for m in mgs:
        m.close()
    for r in rends:
        r.close()
