"""Child process of tests/test_multigpu_ipc.py::test_fine_exchange_after_freed_uncached_allocations (GPU).

Replays the r05 sequence behind the barrier timeouts (profiles/r05_mg_uncached_diag_nokeep.log)
in one process: per case, virtual-rank exchanges over *uncached* memory (GSM_MG_MEM=uncached-ab, the A/B kind
the product refuses; prepared and connected -- the connect's mapping check writes every page -- but no frame is
rendered on it: records read from it can be garbage, r03-r05) plus raw uncached allocations of the exchange
sizes, everything freed, then a fine-grained exchange of the same shape -- whose allocations can land on the
freed uncached ranges.  The fine exchange either refuses at connect (its mapping check) or renders two frames
that are compared with the oracle; barrier timeout 2 s.  Writes {"cases": [{case, refused, timeouts,
bad_rows}]} to argv[1].

usage: python tests/mg_uc_reuse.py OUT.json"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gsm-renderer_amd"), os.path.join(ROOT, "oracle")]
import torch  # noqa: E402

import gsm_amd as gsm  # noqa: E402
import oracle as O  # noqa: E402  (the checker)
from gsm_amd import scenes  # noqa: E402

HIP = C.CDLL("libamdhip64.so")
HIP_UNCACHED = 0x3  # hipDeviceMallocUncached


def raw_uncached(sizes):
    """Allocate, write and free uncached device memory of the given sizes (their ranges become free).
    Returns the HIP status of every allocation (and leaves no error behind for the next HIP call)."""
    ptrs, st = [], []
    for b in sizes:
        p = C.c_void_p()
        rc = HIP.hipExtMallocWithFlags(C.byref(p), C.c_size_t(b), C.c_uint(HIP_UNCACHED))
        st.append(int(rc))
        if rc == 0:
            HIP.hipMemset(p, 0x5A, C.c_size_t(b))
            ptrs.append(p)
    HIP.hipDeviceSynchronize()
    for p in ptrs:
        HIP.hipFree(p)
    HIP.hipDeviceSynchronize()
    HIP.hipGetLastError()
    return st


def frames(world, n, w, h, sh, prec, cams, inp, opts, kind, render=True):
    if kind == "uncached":
        os.environ["GSM_MG_MEM"] = "uncached-ab"
    else:
        os.environ.pop("GSM_MG_MEM", None)
    cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
    rends = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(world)]
    out = {"refused": False, "timeouts": 0, "pix": []}
    pre, mgs = [], []
    try:  # prepare checks (and, failing, replaces) the rank's own allocation; connect checks every mapping
        for k, r in enumerate(rends):
            pre.append(gsm.MultiGpuRenderer.prepare(r, k, world, opts))
        mgs = [m.connect_handles([hd for _, hd in pre]) for m, _ in pre]
    except gsm.RendererError as e:
        if e.status != gsm.Status.DEVICE_NOT_AVAILABLE:
            raise
        out["refused"] = "connect" if len(pre) == world else "prepare"
        for m, _ in pre:
            m.close()
    if mgs and not render:
        for m in mgs:
            m.close()
        mgs = []
    if mgs:
        frame_ptr, _ = mgs[0].frame()
        stream = torch.cuda.current_stream()
        for cam in cams:
            cp = gsm.CameraParams.from_dict(cam)
            for ph in range(4):
                for k, m in enumerate(mgs):
                    m.render_phases([ph], None, None, inp, cp, w, h, gather=True, stream=stream,
                                    gather_target=frame_ptr if k == 0 else None, gather_depth=False)
            torch.cuda.synchronize()
            out["pix"].append(mgs[0].copy_frame(w, h))
        out["timeouts"] = sum(m.status() for m in mgs)
        for m in mgs:
            m.close()
    for r in rends:
        r.close()
    torch.cuda.synchronize()
    return out


def main():
    O.build()
    cases = [(3, 60_000, 1280, 720, 1), (8, 50_000, 640, 360, 0)]
    res = []
    for world, n, w, h, prec in cases:
        sh = 16 if prec else 4
        world_np, harm_np, _ = scenes.gen_scene(n, w, h, sh, prec, seed=78)
        wt = torch.from_numpy(world_np.view(np.uint8).reshape(-1).copy()).cuda()
        ht = torch.from_numpy(harm_np.view(np.uint8).reshape(-1).copy()).cuda()
        inp = gsm.GaussianInput(wt, ht, n, sh)
        cams = [scenes.make_camera(w, h), scenes.orbit_camera(w, h, 5.0)]
        refs = [O.render(world_np, harm_np, sh, c, w, h, max_gaussians=n)["color"] for c in cams]
        opts = gsm.MultiGpuOptions(timeout_ms=2000)
        for rep in range(2):
            uc = frames(world, n, w, h, sh, prec, cams, inp, opts, "uncached", render=False)
            rec = 2 * ((n * 48 + 4095) // 4096 * 4096) + 4096
            alloc = raw_uncached([rec] * world + [w * h * 8, w * h * 2])
            fine = frames(world, n, w, h, sh, prec, cams, inp, opts, "fine")
            bad = [int(np.count_nonzero(np.any(p != r, axis=(1, 2)))) for p, r in zip(fine["pix"], refs)]
            c = {"case": [world, n, w, h, prec, rep], "refused": fine["refused"], "timeouts": fine["timeouts"],
                 "bad_rows": bad, "uncached_refused": uc["refused"], "uncached_timeouts": uc["timeouts"],
                 "raw_alloc_status": alloc}
            detail = []
            for p, r in zip(fine["pix"], refs):  # where and what the wrong pixels are
                rows = np.nonzero(np.any(p != r, axis=(1, 2)))[0]
                if len(rows):
                    y = int(rows[0])
                    xs = np.nonzero(np.any(p[y] != r[y], axis=1))[0]
                    detail.append({"rows": rows[:8].tolist(), "row0_cols": [int(xs.min()), int(xs.max()), int(len(xs))],
                                   "got": p[y, xs[0]].tolist(), "ref": r[y, xs[0]].tolist(),
                                   "byte_off": int(y * w * 8 + xs.min() * 8)})
            if detail:
                c["detail"] = detail
            print(json.dumps(c), flush=True)
            res.append(c)
    with open(sys.argv[1], "w") as f:
        json.dump({"cases": res}, f)


if __name__ == "__main__":
    main()
