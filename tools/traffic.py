"""Per-launch PMC numbers of one kernel from rocprofv3 --pmc passes (tools/gpu_round.sh), raw.

Prints the JSON bench.py reads (--traffic-json): FETCH_SIZE and WRITE_SIZE (KiB per dispatch, the
L2's fabric request counters) and SQ_INSTS_VALU (wave-instructions per dispatch), averaged over
the dispatches.  The counter corrections are bench.py's (roofline "traffic"), calibrated on
MI355X by tools/exp/fetch_calib.hip (profiles/r02_fetch_calibration.json):
  * wide coalesced streams: FETCH_SIZE counts half their bytes (MI355X_MICROARCH.md) -> x2;
  * random gathers of 4 or 16 B: one 64-B FETCH unit per distinct 64-B segment fetched -> x1;
  * WRITE_SIZE exact.
usage: traffic.py PMC_DIR KERNEL_SUBSTRING CONFIG_NAME"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/round/pmc"
kernel = sys.argv[2] if len(sys.argv) > 2 else "k_blend_px"
config = sys.argv[3] if len(sys.argv) > 3 else "cfg2_1m_sh3_1080p_f16"
acc = defaultdict(lambda: defaultdict(list))
for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    with open(path) as f:
        for row in csv.DictReader(f):
            acc[row.get("Kernel_Name", "?")][row["Counter_Name"]].append(float(row["Counter_Value"]))


def mean(cs, name):
    v = cs.get(name)
    return sum(v) / len(v) if v else None


out = {}
# the matching kernel with the most dispatches: a one-frame variant of the same name (the DepthFirst
# blend's walk-statistics instance, k_df_blend_eye<16, true>) is not the frame's kernel
cands = [(len(cs["FETCH_SIZE"]), k) for k, cs in acc.items() if kernel in k and "FETCH_SIZE" in cs and "WRITE_SIZE" in cs]
for _, k in sorted(cands)[-1:]:
    cs = acc[k]
    out = {
        "kernel": k.split("(")[0],
        "config": config,
        "source": "rocprofv3 --pmc passes of bench.py (tools/gpu_round.sh): FETCH_SIZE, WRITE_SIZE and "
                  "SQ_INSTS_VALU each in its own pass",
        "fetch_size_kib": round(mean(cs, "FETCH_SIZE"), 1),
        "write_size_kib": round(mean(cs, "WRITE_SIZE"), 1),
        "valu_insts_per_launch": int(round(mean(cs, "SQ_INSTS_VALU"))) if "SQ_INSTS_VALU" in cs else None,
        "grbm_gui_active": mean(cs, "GRBM_GUI_ACTIVE"),
    }
    # the VALU instruction mix by issue class (SQ_INSTS_VALU_* passes): bench.py prices each class at
    # its measured issue cost (tools/exp/valu_peak.hip) for the mix-weighted roofline_valu
    cls = {n: mean(cs, "SQ_INSTS_VALU_" + n) for n in ("ADD_F16", "MUL_F16", "FMA_F16", "TRANS_F16", "ADD_F32",
                                                      "MUL_F32", "FMA_F32", "TRANS_F32", "INT32", "INT64", "CVT")}
    if all(v is not None for v in cls.values()) and out["valu_insts_per_launch"]:
        mix = {"f16": cls["ADD_F16"] + cls["MUL_F16"] + cls["FMA_F16"], "trans": cls["TRANS_F16"] + cls["TRANS_F32"],
               "f32": cls["ADD_F32"] + cls["MUL_F32"] + cls["FMA_F32"], "int32": cls["INT32"], "int64": cls["INT64"],
               "cvt": cls["CVT"]}
        mix["other"] = max(0.0, out["valu_insts_per_launch"] - sum(mix.values()))
        out["valu_mix_per_launch"] = {k: int(round(v)) for k, v in mix.items()}
print(json.dumps(out, indent=1))
