"""Debug: determinism of the partition kernels in isolation (one renderer, one process, no barriers):
project_partition (k_project_part, k_part_scan, k_part_pack) and render_records (k_records_in ...)
repeated; outputs must be identical every time."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "gsm-renderer_amd")]
import torch
import gsm_amd as gsm
from gsm_amd import scenes
print("rank probe (lane-ordered atomics):", gsm.sort_rank_probe(0), flush=True)
n, w, h, sh, prec = 50_000, 640, 360, 4, 0
wn, hn, cam = scenes.gen_scene(n, w, h, sh, prec, seed=78)
wt = torch.from_numpy(wn.view(np.uint8).reshape(-1).copy()).cuda()
ht = torch.from_numpy(hn.view(np.uint8).reshape(-1).copy()).cuda()
inp = gsm.GaussianInput(wt, ht, n, sh)
cp = gsm.CameraParams.from_dict(cam)
cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
r = gsm.GlobalRenderer(device=0, config=cfg)
rows = [0, 3, 6, 9, 12, 15, 18, 21, 23]
W = 8
send = torch.zeros(n * W * 48, dtype=torch.uint8, device="cuda")
sc = torch.zeros(W, dtype=torch.int32, device="cuda")
base_send = None
bad_pack = 0
for it in range(20):
    send.fill_(0xAB)
    r.project_partition(inp, cp, w, h, 0, n, rows, send, n * W, sc)
    torch.cuda.synchronize()
    tot = int(sc.sum().item())
    s = send[: tot * 48].cpu().numpy()
    if base_send is None:
        base_send = s
    elif not np.array_equal(s, base_send):
        bad_pack += 1
        d = np.nonzero(np.any(s.reshape(-1, 48) != base_send.reshape(-1, 48), axis=1))[0]
        print("pack run", it, "records differ", len(d), d[:6].tolist(), flush=True)
print("pack runs differing:", bad_pack, "records", tot, flush=True)
counts = sc.cpu().numpy().astype(np.int64)
offs = np.concatenate([[0], np.cumsum(counts)])
rend = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(W)]
col = torch.zeros((h, w, 4), dtype=torch.float16, device="cuda")
for d in range(W):
    rend[d].set_tile_rows(rows[d], rows[d + 1])
ref_tc = [None] * W
bad_rec = 0
for it in range(20):
    for d in range(W):
        recs = send[offs[d] * 48: offs[d + 1] * 48]
        rend[d].render_records(col, None, recs, int(counts[d]), w, h)
    torch.cuda.synchronize()
    for d in range(W):
        tc = rend[d].copy_buffer(gsm.BufferId.TILE_COUNTS).view(np.uint32)[: counts[d]].copy()
        if ref_tc[d] is None:
            ref_tc[d] = tc
        elif not np.array_equal(tc, ref_tc[d]):
            bad_rec += 1
            dd = np.nonzero(tc != ref_tc[d])[0]
            print("records_in run", it, "slab", d, "tile counts differ", len(dd), dd[:6].tolist(), flush=True)
print("records_in runs differing:", bad_rec, flush=True)
