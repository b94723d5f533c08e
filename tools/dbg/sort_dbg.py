import os, sys, numpy as np, torch
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [R + "/tests", R + "/oracle", R + "/gsm-renderer_amd"]
import gsm_amd
from golden import make_golden as MG
import test_gpu_parity as T
name = sys.argv[1] if len(sys.argv) > 1 else 'ref_visible_50k_640x360_sh0_f32'
case = MG.scene(name)
r = MG.render(name)
g = T.gpu_render(gsm_amd, torch, case)
gk, rk = g["sorted_keys"], r["sorted_keys"]
gv, rv = g["sorted_values"], r["sorted_values"]
h = r["headers"].reshape(-1, 2)
print("headers equal", np.array_equal(g["headers"], r["headers"]), "unsorted keys equal", np.array_equal(g["keys"], r["keys"]))
bad = []
for t in range(len(h)):
    o, c = h[t]
    if not (np.array_equal(gk[o:o+c], rk[o:o+c]) and np.array_equal(gv[o:o+c], rv[o:o+c])):
        bad.append(t)
print("bad tiles", len(bad), bad[:20], "counts", [int(h[t][1]) for t in bad[:20]])
for t in bad[:2]:
    o, c = h[t]
    print("tile", t, "count", c)
    print(" gpu k", [hex(x) for x in gk[o:o+min(c,12)]])
    print(" ref k", [hex(x) for x in rk[o:o+min(c,12)]])
    print(" gpu v", gv[o:o+min(c,12)].tolist())
    print(" ref v", rv[o:o+min(c,12)].tolist())
