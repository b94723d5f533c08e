"""Debug: dbg2's sequence; on a bad frame, per-rank assignments and an own-target re-render."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "gsm-renderer_amd")]
import torch
import gsm_amd as gsm
import oracle as O
from gsm_amd import scenes
O.build()
cases = [(2, 40_000, 640, 360, 1), (3, 60_000, 1280, 720, 1), (8, 50_000, 640, 360, 0)]
refs = {}
for it in range(3):
    for world, n, w, h, prec in cases:
        sh = 16 if prec else 4
        cams = [scenes.make_camera(w, h), scenes.orbit_camera(w, h, 5.0)]
        key = (world, n, w, h, prec)
        wn, hn, _ = scenes.gen_scene(n, w, h, sh, prec, seed=78)
        if key not in refs:
            refs[key] = [O.render(wn, hn, sh, c, w, h, max_gaussians=n)["color"] for c in cams]
        wt = torch.from_numpy(wn.view(np.uint8).reshape(-1).copy()).cuda()
        ht = torch.from_numpy(hn.view(np.uint8).reshape(-1).copy()).cuda()
        inp = gsm.GaussianInput(wt, ht, n, sh)
        cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
        rends = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(world)]
        pre = [gsm.MultiGpuRenderer.prepare(r, k, world) for k, r in enumerate(rends)]
        mgs = [m.connect_handles([hd for _, hd in pre]) for m, _ in pre]
        fp = mgs[0].frame()[0]
        stream = torch.cuda.current_stream()
        for i, cam in enumerate(cams):
            cp = gsm.CameraParams.from_dict(cam)
            for ph in range(4):
                for k, m in enumerate(mgs):
                    m.render_phases([ph], None, None, inp, cp, w, h, gather=True, stream=stream,
                                    gather_target=fp if k == 0 else None)
            torch.cuda.synchronize()
            got = mgs[0].copy_frame(w, h)
            ref = refs[key][i]
            rows = np.nonzero(np.any(got != ref, axis=(1, 2)))[0]
            info = ""
            if len(rows):
                cnt = [r.counters()["total_assignments"] for r in rends]
                cm = mgs[0].counts().astype(np.int64)
                bad_ex = [m.copy_exchange(4096 + 48 * int(cm[:, k].sum()) + 48 * 64) for k, m in enumerate(mgs)]
                bad_tc = [r.copy_buffer(gsm.BufferId.TILE_COUNTS).view(np.uint32).copy() for r in rends]
                bad_bd = [r.copy_buffer(gsm.BufferId.BOUNDS).view(np.int32).reshape(-1, 4).copy() for r in rends]
                col = torch.full((h, w, 4), float("nan"), dtype=torch.float16, device="cuda")
                for ph in range(4):
                    for k, m in enumerate(mgs):
                        m.render_phases([ph], col, None, inp, cp, w, h, gather=False, stream=stream)
                torch.cuda.synchronize()
                own = col.view(torch.int16).cpu().numpy().view(np.uint16)
                rows_o = np.nonzero(np.any(own != ref, axis=(1, 2)))[0]
                for ph in range(4):
                    for k, m in enumerate(mgs):
                        m.render_phases([ph], None, None, inp, cp, w, h, gather=True, stream=stream,
                                        gather_target=fp if k == 0 else None)
                torch.cuda.synchronize()
                again = mgs[0].copy_frame(w, h)
                cm2 = mgs[0].counts().astype(np.int64)
                good_ex = [m.copy_exchange(len(b)) for m, b in zip(mgs, bad_ex)]
                good_tc = [r.copy_buffer(gsm.BufferId.TILE_COUNTS).view(np.uint32).copy() for r in rends]
                good_bd = [r.copy_buffer(gsm.BufferId.BOUNDS).view(np.int32).reshape(-1, 4).copy() for r in rends]
                for k in range(world):
                    nrec = int(cm[:, k].sum())
                    d = np.nonzero(bad_tc[k][:nrec] != good_tc[k][:nrec])[0]
                    db = np.nonzero(np.any(bad_bd[k][:nrec] != good_bd[k][:nrec], axis=1))[0]
                    print("  rank", k, "tile-count diffs", len(d), d[:8].tolist(), "bad", bad_tc[k][d[:8]].tolist(),
                          "good", good_tc[k][d[:8]].tolist(), "bounds diffs", len(db), flush=True)
                    if len(d):
                        rec = good_ex[k][4096:].reshape(-1, 48)[d[0]].view(np.uint32)
                        print("   record", rec.tolist(), "bounds", good_bd[k][d[0]].tolist(), flush=True)
                for k in range(world):
                    b, g = bad_ex[k], good_ex[k]
                    cb = b[1024:3072].view(np.uint32).reshape(2, 16, 16)
                    cg = g[1024:3072].view(np.uint32).reshape(2, 16, 16)
                    rb = b[4096:].reshape(-1, 48)
                    rg = g[4096:].reshape(-1, 48)
                    nrec = int(cm[:, k].sum())
                    diff = np.nonzero(np.any(rb[:nrec] != rg[:nrec], axis=1))[0]
                    print("  rank", k, "nrec", nrec, int(cm2[:, k].sum()), "count-matrix parity1 equal",
                          bool(np.array_equal(cb[1], cg[1])), "flags", b[:192].view(np.uint32).reshape(3, 16)[:, :world].tolist(),
                          "records differ", len(diff), diff[:5].tolist(), flush=True)
                    if len(diff):
                        i = diff[0]
                        print("   bad ", rb[i].view(np.uint32).tolist(), "\n   good", rg[i].view(np.uint32).tolist(), flush=True)
                rows_a = np.nonzero(np.any(again != ref, axis=(1, 2)))[0]
                info = f" assign {cnt} own-bad {len(rows_o)} again-bad {len(rows_a)} fp {hex(fp)} mem {[hex(h.ctypes.data) for h in []]}"
            print(it, key, "frame", i, "bad rows", len(rows), rows[:2].tolist(), info, flush=True)
        for m in mgs:
            m.close()
        for r in rends:
            r.close()
        del wt, ht
