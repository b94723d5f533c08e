"""Per-launch HBM traffic of the blend kernel from rocprofv3 PMC passes (tools/gpu_round.sh).

MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE come from the L2's fabric request
counters; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so it is doubled;
WRITE_SIZE is exact.  Both are in KiB per dispatch.  Prints the JSON bench.py reads."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/round/pmc"
kernel = sys.argv[2] if len(sys.argv) > 2 else "k_blend_px"          # kernel name substring
config = sys.argv[3] if len(sys.argv) > 3 else "cfg2_1m_sh3_1080p_f16"
acc = defaultdict(lambda: defaultdict(list))
for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    with open(path) as f:
        for row in csv.DictReader(f):
            acc[row.get("Kernel_Name", "?")][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {}
for k, cs in acc.items():
    if kernel not in k or "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
        continue
    f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
    w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
    out = {
        "kernel": k.split("(")[0],
        "config": config,
        "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (tools/gpu_round.sh)",
        "fetch_size_kb": round(f, 1),
        "write_size_kb": round(w, 1),
        "correction": "FETCH_SIZE x2 (gfx950 counts half of wide reads), WRITE_SIZE exact",
        "blend_hbm_bytes_per_launch": int(round((2 * f + w) * 1024)),
        "blend_valu_insts_per_launch": (int(round(sum(cs["SQ_INSTS_VALU"]) / len(cs["SQ_INSTS_VALU"])))
                                        if "SQ_INSTS_VALU" in cs else None),
        "note": "includes each workgroup's 128 KiB exp-table load and the re-reads of a tile's list by "
                "every unit of the tile; Infinity-Cache hits are counted by these fabric counters",
    }
print(json.dumps(out, indent=1))
